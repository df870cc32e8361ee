// bank_probe.hip -- does the VGPR bank of a VOP3's source operands change its
// issue rate on gfx950?  Each variant is a loop of 32 v_bitop3_b32 with
// fixed registers (inline asm), run at full occupancy; prints ns per
// instruction per SIMD.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP32(x) REP8(x) REP8(x) REP8(x) REP8(x)

template <int V>
__global__ __launch_bounds__(256) void probe(int iters, unsigned *out) {
  unsigned r;
  if constexpr (V == 0) {  // sources v44, v48, v52: one bank
    asm volatile(
        "v_mov_b32 v44, 1\n v_mov_b32 v48, 2\n v_mov_b32 v52, 3\n s_mov_b32 s40, %1\n"
        "1:\n" REP32("v_bitop3_b32 v40, v44, v48, v52 bitop3:0x96\n")
        "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n"
        : "=v"(r) : "s"(iters) : "v40", "v44", "v48", "v52", "s40", "scc");
  } else if constexpr (V == 1) {  // sources v41, v42, v43: three banks
    asm volatile(
        "v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\n s_mov_b32 s40, %1\n"
        "1:\n" REP32("v_bitop3_b32 v40, v41, v42, v43 bitop3:0x96\n")
        "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n"
        : "=v"(r) : "s"(iters) : "v40", "v41", "v42", "v43", "s40", "scc");
  } else if constexpr (V == 2) {  // two of three in one bank
    asm volatile(
        "v_mov_b32 v41, 1\n v_mov_b32 v45, 2\n v_mov_b32 v43, 3\n s_mov_b32 s40, %1\n"
        "1:\n" REP32("v_bitop3_b32 v40, v41, v45, v43 bitop3:0x96\n")
        "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n"
        : "=v"(r) : "s"(iters) : "v40", "v41", "v45", "v43", "s40", "scc");
  } else if constexpr (V == 3) {  // dependent chain, distinct banks
    asm volatile(
        "v_mov_b32 v40, 0\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\n s_mov_b32 s40, %1\n"
        "1:\n" REP32("v_bitop3_b32 v40, v40, v42, v43 bitop3:0x96\n")
        "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n"
        : "=v"(r) : "s"(iters) : "v40", "v42", "v43", "s40", "scc");
  } else if constexpr (V == 4) {  // v_alignbit, two sources one bank
    asm volatile(
        "v_mov_b32 v44, 1\n v_mov_b32 v48, 2\n s_mov_b32 s40, %1\n"
        "1:\n" REP32("v_alignbit_b32 v40, v44, v48, 31\n")
        "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n"
        : "=v"(r) : "s"(iters) : "v40", "v44", "v48", "s40", "scc");
  } else if constexpr (V == 5) {  // v_alignbit, distinct banks
    asm volatile(
        "v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n s_mov_b32 s40, %1\n"
        "1:\n" REP32("v_alignbit_b32 v40, v41, v42, 31\n")
        "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n"
        : "=v"(r) : "s"(iters) : "v40", "v41", "v42", "s40", "scc");
  } else if constexpr (V == 6) {  // plain VOP2 v_xor_b32
    asm volatile(
        "v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n s_mov_b32 s40, %1\n"
        "1:\n" REP32("v_xor_b32 v40, v41, v42\n")
        "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n"
        : "=v"(r) : "s"(iters) : "v40", "v41", "v42", "s40", "scc");
  } else if constexpr (V == 7) {  // DPP wave_ror
    asm volatile(
        "v_mov_b32 v41, 1\n s_mov_b32 s40, %1\n s_nop 4\n"
        "1:\n" REP32("v_mov_b32_dpp v40, v41 wave_ror:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n")
        "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n"
        : "=v"(r) : "s"(iters) : "v40", "v41", "s40", "scc");
  } else if constexpr (V == 8) {  // DPP row_shr:1 (within a row of 16)
    asm volatile(
        "v_mov_b32 v41, 1\n s_mov_b32 s40, %1\n s_nop 4\n"
        "1:\n" REP32("v_mov_b32_dpp v40, v41 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n")
        "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n"
        : "=v"(r) : "s"(iters) : "v40", "v41", "s40", "scc");
  } else if constexpr (V == 9) {  // v_xor_b32 with DPP wave_ror on src0
    asm volatile(
        "v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n s_mov_b32 s40, %1\n s_nop 4\n"
        "1:\n" REP32("v_xor_b32_dpp v40, v41, v42 wave_ror:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n")
        "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n"
        : "=v"(r) : "s"(iters) : "v40", "v41", "v42", "s40", "scc");
  } else if constexpr (V == 10) {  // v_bitop3 with one SGPR-free literal-free, sources v41 v42 and v41 again
    asm volatile(
        "v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n s_mov_b32 s40, %1\n"
        "1:\n" REP32("v_bitop3_b32 v40, v41, v42, v41 bitop3:0x96\n")
        "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n"
        : "=v"(r) : "s"(iters) : "v40", "v41", "v42", "s40", "scc");
  } else if constexpr (V == 11) {  // ds_bpermute throughput (LDS pipe)
    asm volatile(
        "v_mov_b32 v41, 1\n v_lshlrev_b32 v42, 2, v41\n s_mov_b32 s40, %1\n"
        "1:\n" REP32("ds_bpermute_b32 v40, v42, v41\n")
        "s_waitcnt lgkmcnt(0)\n"
        "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n"
        : "=v"(r) : "s"(iters) : "v40", "v41", "v42", "s40", "scc");
  }
  if (r == 0x12345678u) out[0] = r;
}

static const char *names[] = {"bitop3_1bank",  "bitop3_3banks", "bitop3_2in1bank", "bitop3_chain",
                              "alignbit_1bank", "alignbit_2banks", "xor_vop2",     "dpp_wave_ror",
                              "dpp_row_shr",   "xor_dpp_wave_ror", "bitop3_repeat", "ds_bpermute"};

template <int V>
void run(int cus) {
  unsigned *out;
  (void)hipMalloc(&out, 4);
  const int iters = 4000, blocks = cus * 8;  // 8 blocks x 4 waves = 32 waves/CU = 8/SIMD
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int w = 0; w < 2; ++w) probe<V><<<blocks, 256>>>(iters, out);
  (void)hipEventRecord(a);
  const int reps = 5;
  for (int w = 0; w < reps; ++w) probe<V><<<blocks, 256>>>(iters, out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  // instructions per SIMD: waves per SIMD (8) x iters x 32
  const double per_simd = 8.0 * iters * 32 * reps;
  std::printf("{\"variant\": \"%s\", \"ns_per_instr_per_simd\": %.4f, \"clk_at_2.4GHz\": %.3f}\n", names[V],
              ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.4);
  (void)hipFree(out);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  run<0>(cus); run<1>(cus); run<2>(cus); run<3>(cus); run<4>(cus); run<5>(cus);
  run<6>(cus); run<7>(cus); run<8>(cus); run<9>(cus); run<10>(cus); run<11>(cus);
  return 0;
}
