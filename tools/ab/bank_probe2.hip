// bank_probe2.hip -- issue cost of the shift/permute candidates for the
// 64-bit row rotate and the column exchange; same harness as bank_probe.hip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <utility>
#define REP8(x) x x x x x x x x
#define REP32(x) REP8(x) REP8(x) REP8(x) REP8(x)
template <int V> __global__ __launch_bounds__(256) void probe(int iters, unsigned *out) {
  unsigned r = 0;
  if constexpr (V == 0) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\ns_mov_b32 s41, 31\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_alignbit_b32 v40, v41, v42, s41\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 1) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\nv_mov_b32 v43, 31\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_alignbit_b32 v40, v41, v42, v43\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 2) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_alignbyte_b32 v40, v41, v42, 1\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 3) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_lshlrev_b32 v40, 1, v41\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 4) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_lshrrev_b32 v40, 31, v41\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 5) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_lshl_or_b32 v40, v41, 1, v42\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 6) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_lshlrev_b64 v[44:45], 1, v[42:43]\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 7) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\nv_mov_b32 v46, 0\n v_mov_b32 v47, 0\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_lshl_add_u64 v[44:45], v[42:43], 1, v[46:47]\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 8) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\nv_mov_b32 v43, 0x05040100\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_perm_b32 v40, v41, v42, v43\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 9) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\nv_mov_b32 v43, 3\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_bfi_b32 v40, v41, v42, v43\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 10) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\nv_mov_b32 v43, 3\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_add3_u32 v40, v41, v42, v43\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 11) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\nv_mov_b32 v43, 3\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_bitop3_b16 v40, v41, v42, v43 bitop3:0x96\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 12) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\nv_mov_b32 v46, 0\n v_mov_b32 v47, 0\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_pk_mov_b32 v[44:45], v[42:43], v[46:47] op_sel:[1,0]\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 13) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_mov_b64 v[44:45], v[42:43]\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 14) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\ns_mov_b32 s41, 31\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_xor_b32_e64 v40, s41, v42\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 15) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\ns_mov_b32 s41, 31\n v_mov_b32 v43, 3\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_bitop3_b32 v40, s41, v42, v43 bitop3:0x96\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 16) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_lshlrev_b16 v40, 1, v41\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 17) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_pk_lshlrev_b16 v40, 1, v41\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 18) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_bfe_u32 v40, v41, 1, 31\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 19) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\ns_mov_b64 vcc, -1\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_cndmask_b32 v40, v41, v42, vcc\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 20) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\nv_mov_b32 v44, 1\n v_mov_b32 v45, 2\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_permlane32_swap_b32 v44, v45\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if constexpr (V == 21) asm volatile("v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\nv_mov_b32 v44, 1\n v_mov_b32 v45, 2\n s_mov_b32 s40, %1\n s_nop 4\n 1:\n" REP32("v_permlane16_swap_b32 v44, v45\n") "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v40\n" : "=v"(r) : "s"(iters) : "v40","v41","v42","v43","v44","v45","v46","v47","s40","s41","vcc","scc");
  if (r == 0x12345678u) out[0] = r;
}
static const char *names[] = {"alignbit_sgpr_shift", "alignbit_vgpr_shift", "alignbyte", "lshlrev_b32_vop2", "lshrrev_b32_vop2", "lshl_or_b32", "lshlrev_b64", "lshl_add_u64", "perm_b32", "bfi_b32", "add3_u32", "bitop3_b16", "pk_mov_b32", "mov_b64", "xor_b32_vop3_sgpr", "bitop3_sgpr_src", "lshlrev_b16", "pk_lshlrev_b16", "bfe_u32", "cndmask", "permlane32_swap", "permlane16_swap"};
template <int V> void run(int cus) {
  unsigned *out; (void)hipMalloc(&out, 4);
  const int iters = 4000, blocks = cus * 8, reps = 5;
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (int w = 0; w < 2; ++w) probe<V><<<blocks, 256>>>(iters, out);
  (void)hipEventRecord(a);
  for (int w = 0; w < reps; ++w) probe<V><<<blocks, 256>>>(iters, out);
  (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  const double per_simd = 8.0 * iters * 32 * reps;
  std::printf("{\"variant\": \"%s\", \"ns_per_instr_per_simd\": %.4f}\n", names[V], ms * 1e6 / per_simd);
  (void)hipFree(out);
}
template <int... V> void run_all(int cus, std::integer_sequence<int, V...>) { (run<V>(cus), ...); }
int main() {
  hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0);
  run_all(p.multiProcessorCount, std::make_integer_sequence<int, 22>{});
  return 0;
}
