"""CPU: pin the oracle (C restatement) against the reference's golden vectors.

The fixtures in tests/golden/ were produced by the reference's OWN code
(tests/golden/make_golden.py, via oracle/_ref).  Where oracle/_ref is present
(build container and GPU box) the restatement is also compared with the live
reference on fresh seeded inputs.
"""
import json
import os
import sys

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLD, name))  # allow_pickle=False (default)


@pytest.fixture(scope="module")
def meta():
    with open(os.path.join(GOLD, "golden.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("form", [0, 1, 2])
def test_random_step_golden(port, form):
    g = load("random_step.npz")
    assert (port.step_batch(g["input"], 1, formulation=form) == g["step1"]).all()
    assert (port.step_batch(g["input"], 1024, formulation=form) == g["step1024"]).all()


def test_edge_cases_golden(port, meta):
    g = load("edge_cases.npz")
    for k in g["gens"]:
        got = port.step_batch(g["input"], int(k))
        bad = [meta["edge_cases"]["names"][i] for i in np.nonzero((got != g[f"step{k}"]).any(1))[0]]
        assert not bad, f"gen {k}: {bad}"


def test_edge_case_semantics(port, meta):
    """Known behaviour of the fixtures themselves (not just self-consistency)."""
    g = load("edge_cases.npz")
    names = meta["edge_cases"]["names"]
    x = dict(zip(names, g["input"]))
    s1 = dict(zip(names, g["step1"]))
    assert not s1["all_on"].any() and not s1["checkerboard"].any() and not s1["empty"].any()
    assert (dict(zip(names, g["step2"]))["blinker_both_seams"] == x["blinker_both_seams"]).all()
    assert (s1["block_corners"] == x["block_corners"]).all()
    # glider: +1 column, +1 row every 4 generations, through both seams
    s4 = dict(zip(names, g["step4"]))
    for nm in ("glider", "glider_col_seam", "glider_row_seam", "glider_corner"):
        moved = np.roll(x[nm], 1)
        moved = np.array([((int(w) << 1) | (int(w) >> 63)) & (2**64 - 1) for w in moved], np.uint64)
        assert (s4[nm] == moved).all(), nm
    assert (dict(zip(names, g["step256"]))["glider"] == x["glider"]).all()


def test_rpentomino_known_answer(port, meta):
    g = load("rpentomino.npz")
    r = port.parse("b2o$2o$bo!")
    assert (r == g["initial"]).all()
    s, trace = r.copy(), [int(port.pop(r[None])[0])]
    for _ in range(1103):
        s = port.step_batch(s[None], 1)[0]
        trace.append(int(port.pop(s[None])[0]))
    assert trace == g["pop_trace"].tolist()
    assert (s == g["final"]).all()
    assert trace[1103] == 113 and meta["rpentomino"]["final_pop"] == 113


def test_randomstate_kat(port):
    """StepAltTest.cpp:5-13 on the reference's own RandomState() draws."""
    g = load("randomstate_kat.npz")
    for form in (0, 1, 2):
        assert (port.step_batch(g["input"], 1, formulation=form) == g["step"]).all()
    # RandomState shape: row 61 always on, rows 62-63 off (LifeAPI.hpp:18-23)
    assert ((g["input"] >> np.uint64(61)) == 1).all()
    for u in range(g["neighbour_count"].shape[0]):
        assert (port.neighbour_count(g["input"][u]) == g["neighbour_count"][u]).all()


def test_contains_golden(port):
    g = load("contains.npz")
    got = [port.contains(g["states"][u], g["wanted"], g["unwanted"]) for u in range(64)]
    assert np.array(got, dtype=np.uint8).tolist() == g["contains"].tolist()
    assert g["contains"][:8].all() and not g["contains"][8:16].any()


def test_digest_config3_golden(port, meta):
    """Full config-3 workload (64K x 1024 gens) digest matches the reference's."""
    d = meta["digests"]["config3"]
    x = port.fill(d["universes"], d["seed"])
    assert f"{port.digest(port.hashes(x)):016x}" == d["input_digest"]
    out = port.step_batch(x, d["generations"], nthreads=8)
    assert f"{port.digest(port.hashes(out)):016x}" == d["output_digest"]
    assert int(port.pop(out).astype(np.uint64).sum()) == d["output_pop_total"]


def test_digest_config2_input(port, meta):
    d = meta["digests"]["config2"]
    x = port.fill(d["universes"], d["seed"])
    assert f"{port.digest(port.hashes(x)):016x}" == d["input_digest"]
    out = port.step_batch(x, 1, nthreads=4)
    assert f"{port.digest(port.hashes(out)):016x}" == d["output_digest"]
    assert int(port.pop(out).astype(np.uint64).sum()) == d["output_pop_total"]


def test_shard_digests_additive(port, meta):
    """Config-4 sharding: shard digests (first_universe offsets) add to the global one."""
    d = meta["digests"]["config4"]
    k = 3
    x = port.fill(4096, d["seed"], first_universe=k << 21)
    h = port.hashes(x)
    whole = port.digest(h, k << 21)
    parts = (port.digest(h[:1000], k << 21) + port.digest(h[1000:], (k << 21) + 1000)) % 2**64
    assert whole == parts


def test_parse_semantics(port):
    r = port.parse("x = 3, y = 3, rule = B3/S23\nb2o$2o$bo!")
    assert (r == port.parse("b2o$2o$bo!")).all()
    assert port.parse("o$$o!")[0] == 0b101       # bare '$' counts as 1 (Parsing.hpp:161-162)
    assert port.parse("3o!")[2] == 1
    with pytest.raises(ValueError):
        port.parse("65bo!")


def test_counts_golden(port):
    """NeighbourCount (NeighbourCount.hpp:40-70) and InteractionCountsAndNext
    (LifeAPI.hpp:997-1040) planes vs the reference-generated fixture."""
    g = load("counts.npz")
    for u in range(g["input"].shape[0]):
        assert (port.neighbour_count(g["input"][u]) == g["neighbour_count"][u]).all()
        assert (port.interaction_counts(g["input"][u]) == g["interaction_counts"][u]).all()
    # the 'next' plane is Step()
    assert (g["interaction_counts"][:, 3] == port.step_batch(g["input"], 1)).all()


def test_weld_golden(port):
    """LifeWeld::Step (LifeWeld.hpp:169-186) vs the reference-generated
    fixture; the FromRequired welds of LifeWeldTest.cpp:19-33 are invariant."""
    g = load("weld.npz")
    assert (port.weld_step(g["input"], 1) == g["step1"]).all()
    assert (port.weld_step(g["input"], 7) == g["step7"]).all()
    k = int(g["n_required"])
    assert (g["step1"][:k] == g["input"][:k]).all() and g["input"][:k, 64:].any()


def test_weld_equals_reference_live(port, ref):
    w = port.fill(50 * 4, seed=7171).reshape(50, 256)
    w[:, 64:] &= port.fill(150, seed=7172).reshape(50, 192)
    assert (port.weld_step(w, 3) == ref.weld_step(w, 3)).all()


def test_refined_truth_table_fixture(port, meta):
    """Config 5: the fragment's truth table fixture and the harness outputs."""
    tt = port.refined_truth_table()
    assert tt.shape == (3, 1 << 16)
    assert [int(v) for v in tt.sum(axis=1)] == meta["unknown_step_refined"]["ones_per_output"]
    g = load("refined_step.npz")
    assert (port.refined_step(g["input"]) == g["output"]).all()


@pytest.mark.parametrize("inc,ttfile", [("refined_circuit.inc", "unknown_step_refined_tt.npz"),
                                         ("stable_count_circuit.inc", "stable_count_tt.npz"),
                                         ("stable_signal_circuit.inc", "stable_signal_tt.npz"),
                                         ("stable_vulnerable_circuit.inc", "stable_vulnerable_tt.npz")])
def test_generated_circuit_is_the_table(inc, ttfile):
    """A generated bitop3 network (lifeapi_amd/csrc/*.inc), simulated on every
    input combination, is exactly the reference fragment's truth table -- on
    every row, or, for a network generated on the reachable rows
    (tools/cgp_stable.py, its header says so), on every row that
    NeighbourCount-derived inputs can take (test_reachable_rows_cover_every_
    neighbourhood checks that set)."""
    import re
    d = load(ttfile)
    tt = d["tt"].astype(bool)
    nin = tt.shape[1].bit_length() - 1
    src = open(os.path.join(os.path.dirname(GOLD), "..", "lifeapi_amd", "csrc", inc)).read()
    idx = np.arange(1 << nin, dtype=np.uint32)
    val = {f"x[{i}]": ((idx >> i) & 1).astype(bool) for i in range(nin)}
    A, B, C = 0xF0, 0xCC, 0xAA
    for tab, a, b, c, name in [(int(m[1], 16), m[2], m[3], m[4], m[0]) for m in
                               re.findall(r"const T (t\d+) = lut3<0x([0-9A-F]{2})>\(([^,]+), ([^,]+), ([^)]+)\);", src)]:
        va, vb, vc = val[a], val[b], val[c]
        out = np.zeros(1 << nin, bool)
        for bit in range(8):
            if (tab >> bit) & 1:
                out |= (va == bool((A >> bit) & 1)) & (vb == bool((B >> bit) & 1)) & (vc == bool((C >> bit) & 1))
        val[name] = out
    outs = []
    for nm in (str(s) for s in d["outputs"]):
        m = re.search(rf"\b{nm} = (~(t\d+)|(t\d+|x\[\d+\]));", src)
        outs.append(~val[m[2]] if m[2] else val[m[3]])
    got = np.stack(outs)
    if "reachable_rows" in src:
        sys.path.insert(0, os.path.join(os.path.dirname(GOLD), "..", "tools"))
        from cgp_stable import reachable_rows
        rows = reachable_rows(inc.split("_")[1])
        assert (got[:, rows] == tt[:, rows]).all()
    else:
        assert (got == tt).all()


def _inclusive_count(plane: np.ndarray) -> np.ndarray:
    """NeighbourCount (NeighbourCount.hpp:40-70) per cell of a (64, 64) bool
    plane on the torus: the 3x3 block's population, centre included"""
    p = plane.astype(np.int64)
    return sum(np.roll(np.roll(p, dx, 0), dy, 1) for dx in (-1, 0, 1) for dy in (-1, 0, 1))


def test_reachable_rows_cover_every_neighbourhood():
    """The care sets of the resynthesised LifeStable networks
    (tools/cgp_stable.py reachable_rows) contain every input row the passes
    form from real planes: random state / unknown / option planes of many
    densities, state and unknown overlapping too, every cell of every board
    (the kernels compute the same counts, stable_kernels.hpp)."""
    sys.path.insert(0, os.path.join(os.path.dirname(GOLD), "..", "tools"))
    from cgp_stable import reachable_rows
    care = {k: set(reachable_rows(k).tolist()) for k in ("count", "signal", "vulnerable")}
    rng = np.random.default_rng(2024)

    def rowint(cols):
        return sum(c.astype(np.int64) << i for i, c in enumerate(cols))

    def bits(v, hi):
        return [(v >> k) & 1 for k in range(hi, -1, -1)]
    seen = {k: set() for k in care}
    for dens_s, dens_u in [(0.1, 0.1), (0.5, 0.5), (0.9, 0.05), (0.05, 0.9), (0.3, 0.0), (0.0, 0.3), (0.7, 0.7)]:
        for _ in range(3):
            st = rng.random((64, 64)) < dens_s
            un = rng.random((64, 64)) < dens_u
            opt = [rng.random((64, 64)) < 0.5 for _ in range(8)]
            off = ~un & ~st
            on_c, off_c = _inclusive_count(st), _inclusive_count(off)
            m_c, u_c = _inclusive_count(st | un), _inclusive_count(un)
            r = rowint(bits(on_c % 8, 2) + bits(off_c, 3) + [st, off])
            seen["count"] |= set(r.ravel().tolist())
            r = rowint(opt + bits(on_c % 8, 2) + bits(m_c, 3) + [st, un])
            seen["signal"] |= set(r.ravel().tolist())
            r = rowint(opt + bits(on_c % 8, 2) + bits(u_c, 3))
            seen["vulnerable"] |= set(r.ravel().tolist())
    for k in care:
        assert seen[k] <= care[k], k
        assert len(seen[k]) > len(care[k]) // 10  # the sample reaches a good part of the set


def test_rule3_network_truth():
    """The 7-LUT network of k_step RULE 3 (tables parsed from the kernel
    source), evaluated on all 512 3x3 neighbourhoods, is B3/S23 on the
    inclusive count (LifeAPI.hpp:1251-1252: count 3, or 4 with the centre)."""
    import re
    src = open(os.path.join(os.path.dirname(GOLD), "..", "lifeapi_amd", "csrc", "device.hpp")).read()
    t = {k: int(v, 16) for k, v in re.findall(r"\b(kT[123]) = (?:0x)?([0-9A-Fa-f]+)", src)}
    assert set(t) == {"kT1", "kT2", "kT3"}

    def lut(tab, x, y, z):
        return (tab >> ((x << 2) | (y << 1) | z)) & 1

    for bits in range(512):
        n = [(bits >> i) & 1 for i in range(9)]      # n[3*col + row], col 0 = left
        a = n[4]
        cnt = sum(n)
        h = [n[r] + n[3 + r] + n[6 + r] for r in range(3)]
        sa, sb = sum(x & 1 for x in h), sum(x >> 1 for x in h)
        s0, s1, s2, s3 = int(sa <= 1), int(sa in (1, 2)), int(sb <= 1), int(sb in (0, 2))
        t1 = lut(t["kT1"], s0, s1, a)
        t2 = lut(t["kT2"], s2, a, t1)
        assert lut(t["kT3"], s1, s3, t2) == int(cnt == 3 or (a == 1 and cnt == 4)), bits


def test_net6_truth():
    """The 6-LUT tail life_tail6 (gates and tables parsed from device.hpp)
    behind the h-layer h0 = xor3, h1 = maj of each row, on all 512 3x3
    neighbourhoods: B3/S23 on the inclusive count (LifeAPI.hpp:1196-1216)."""
    import re
    src = open(os.path.join(os.path.dirname(GOLD), "..", "lifeapi_amd", "csrc", "device.hpp")).read()
    tabs = {"kMaj": 0xE8, "kNae": 0x7E, "kXor3": 0x96}
    tabs.update({k: int(v, 16) for k, v in re.findall(r"\b(kN[146]) = 0x([0-9A-Fa-f]+)", src)})
    assert set(tabs) == {"kMaj", "kNae", "kXor3", "kN1", "kN4", "kN6"}
    body = src[src.index("uint32_t life_tail6("):]
    body = body[:body.index("\n}\n")]
    gates = re.findall(r"const uint32_t (g\d) = lut3<(\w+)>\((\w+), (\w+), (\w+)\);", body)
    ret = re.search(r"return lut3<(\w+)>\((\w+), (\w+), (\w+)\);", body)
    assert len(gates) == 5 and ret

    def lut(tab, x, y, z):
        return (tab >> ((x << 2) | (y << 1) | z)) & 1

    for bits in range(512):
        n = [(bits >> i) & 1 for i in range(9)]      # n[3*col + row], col 0 = left
        a, cnt = n[4], sum(n)
        rows = [(n[r], n[3 + r], n[6 + r]) for r in range(3)]
        v = {"a": a}
        for nm, r in (("u", 0), ("", 1), ("d", 2)):
            v["h0" + nm] = lut(0x96, *rows[r])
            v["h1" + nm] = lut(0xE8, *rows[r])
        for g, tab, x, y, z in gates:
            v[g] = lut(tabs[tab], v[x], v[y], v[z])
        got = lut(tabs[ret[1]], v[ret[2]], v[ret[3]], v[ret[4]])
        assert got == int(cnt == 3 or (a == 1 and cnt == 4)), bits


def test_weld_tail_truth():
    """The 10-gate LifeWeld tail of k_weld_split (weld_tail, stencil_kernels.hpp:
    gates and tables parsed from the source) behind the h-layer, on all 512
    neighbourhoods x 8 frozen counts, against LifeWeld::Step's adder chain and
    rule (LifeWeld.hpp:169-186: count bits 2..0 + frozen, mod 8)."""
    import re
    src = open(os.path.join(os.path.dirname(GOLD), "..", "lifeapi_amd", "csrc", "stencil_kernels.hpp")).read()
    tabs = {"kMaj": 0xE8, "kXor3": 0x96}
    tabs.update({k: int(v, 16) for k, v in re.findall(r"\b(kW\d) = 0x([0-9A-Fa-f]+)", src)})
    body = src[src.index("uint32_t weld_tail("):]
    body = body[:body.index("\n}\n")]
    gates = re.findall(r"const uint32_t (w\d) = lut3<(\w+)>\((\w+), (\w+), (\w+)\);", body)
    ret = re.search(r"return lut3<(\w+)>\((\w+), (\w+), (\w+)\);", body)
    assert len(gates) == 9 and ret

    def lut(tab, x, y, z):
        return (tab >> ((x << 2) | (y << 1) | z)) & 1

    for bits in range(512):
        n = [(bits >> i) & 1 for i in range(9)]      # n[3*col + row], col 0 = left
        a, cnt = n[4], sum(n)
        rows = [(n[r], n[3 + r], n[6 + r]) for r in range(3)]
        for fz in range(8):
            v = {"a": a, "f0": fz & 1, "f1": (fz >> 1) & 1, "f2": fz >> 2}
            for nm, r in (("u", 0), ("", 1), ("d", 2)):
                v["h0" + nm] = lut(0x96, *rows[r])
                v["h1" + nm] = lut(0xE8, *rows[r])
            for g, tab, x, y, z in gates:
                v[g] = lut(tabs[tab], v[x], v[y], v[z])
            got = lut(tabs[ret[1]], v[ret[2]], v[ret[3]], v[ret[4]])
            t = ((cnt & 7) + fz) & 7
            s0, s1, s2 = t & 1, (t >> 1) & 1, t >> 2
            assert got == (s0 ^ s2) & (s1 ^ s2) & (a | s0), (bits, fz)


def test_stable_vulnerable_golden(port):
    """LifeStable::Vulnerable (LifeStable.hpp:366-412) vs the reference's output."""
    g = load("stable.npz")
    got = port.stable_vulnerable(g["input"])
    assert (got == g["vulnerable"]).all() and g["vulnerable"].any()


def test_stable_passes_golden(port):
    """LifeStable passes (LifeStable.hpp:526-729) vs the reference-generated
    fixture: every plane and the PropagateResult flags, all five passes."""
    g = load("stable.npz")
    for w, name in enumerate(port.STABLE_PASSES):
        out, fl = port.stable_pass(g["input"], w)
        assert (out == g[name]).all(), name
        assert (fl == g[name + "_flags"]).all(), name
    assert (g["propagate_flags"] & 1).sum() >= 5  # some candidates stay consistent


# ---- live reference (present where oracle/_ref was built) ----

def test_port_equals_reference_live(port, ref):
    for seed, mode in ((101, 0), (102, 1)):
        x = port.fill(3000, seed, mode=mode)
        for gens in (1, 7):
            assert (port.step_batch(x, gens) == ref.step_batch(x, gens)).all()
    x = port.fill(200, 103)
    assert (ref.step_alt(x) == port.step_batch(x, 1, formulation=1)).all()
    assert (ref.step_nc(x) == port.step_batch(x, 1, formulation=2)).all()
    for u in range(20):
        assert (ref.neighbour_count(x[u]) == port.neighbour_count(x[u])).all()


def test_reference_search_loop_equals_port(port, ref):
    """ref_shim.cpp's ref_step_contains_batch (the reference's Step() then
    Contains(LifeTarget) per generation) against the port's per-generation
    loop, with planted still-life hits; it is what the config-3 search-loop
    golden digests come from"""
    w, u = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
    w[10] = w[11] = np.uint64(3 << 40)
    for c in (9, 10, 11, 12):
        u[c] = np.uint64(15 << 39)
    u &= ~w
    x = port.fill(300, seed=707) & port.fill(300, seed=708) & port.fill(300, seed=709)
    clear = np.zeros(64, np.uint64)
    clear[2:20] = np.uint64(0x3FFFF << 32)             # an empty 18 x 18 region around the target
    x[::5] = (x[::5] & ~clear) | w
    first, fin = ref.step_contains_batch(x, w, u, 13, nthreads=2)
    exp, s = np.zeros(300, np.uint32), x.copy()
    for g in range(1, 14):
        s = port.step_batch(s, 1)
        hit = np.array([port.contains(s[k], w, u) for k in range(300)])
        exp[(exp == 0) & hit] = g
    assert (first == exp).all() and (fin == s).all()
    assert (exp > 0).sum() >= 60


def test_reference_random_state_shape(ref, port):
    rs = np.stack([ref.random_state() for _ in range(64)])
    assert ((rs >> np.uint64(61)) == 1).all()
    assert (port.step_batch(rs, 1) == ref.step_batch(rs, 1)).all()


def test_counts_equal_reference_live(port, ref):
    x = port.fill(100, seed=4343)
    for u in range(100):
        assert (port.interaction_counts(x[u]) == ref.interaction_counts(x[u])).all()


def test_refined_oracle_equals_reference_fragment(port, ref):
    x = port.fill(200 * 11, seed=909).reshape(200, 11 * 64)
    x[:100, :64] &= port.fill(100, seed=1)           # sparser stable states
    assert (port.refined_step(x) == ref.refined_step(x)).all()


def test_parse_equals_reference(port, ref):
    for rle in ("b2o$2o$bo!", "bo$2bo$3o!", "2b2o$bobo$bo$2o!", "x = 1\n3o$b2o3$o!", "o2$3bo!"):
        assert (port.parse(rle) == ref.parse(rle)).all(), rle


def _blob(text, offs, u):
    return text[int(offs[u]):int(offs[u + 1])].tobytes().decode()


def test_rle_io_golden(port):
    """LifeState::RLE() / Parse (Parsing.hpp:8-63,143-204) vs the reference-
    generated fixture: every state's RLE, every tricky parse case."""
    g = load("rle.npz")
    for u, s in enumerate(g["states"]):
        assert port.rle(s) == _blob(g["rle_text"], g["rle_offsets"], u), u
    for u, want in enumerate(g["parsed"]):
        assert (port.parse(_blob(g["parse_text"], g["parse_offsets"], u)) == want).all(), u


def test_rle_parse_round_trip(port):
    """Parse(RLE(s)) is s moved by (32, 32): RLE prints from x = y = 32."""
    x = port.fill(16, seed=31)
    x[8:] &= port.fill(8, seed=32) & port.fill(8, seed=33)
    for s in x:
        back = port.parse(port.rle(s))
        want = np.roll(s, 32)
        want = np.array([((int(w) << 32) | (int(w) >> 32)) & (2**64 - 1) for w in want], np.uint64)
        assert (back == want).all()


def test_rle_equals_reference(port, ref):
    x = port.fill(24, seed=41)
    x[8:16] &= port.fill(8, seed=42) & port.fill(8, seed=43)
    x[16:] = 0
    x[16:, 5] = np.uint64(1) << np.arange(8, dtype=np.uint64) * np.uint64(7)
    for s in x:
        assert port.rle(s) == ref.rle(s)


def test_prelude_build_matches_minimal_recipe(ref, port):
    """The reference shim built with ref_prelude.hpp (`#define constexpr`
    forced into every translation unit) against the same shim built by
    SURVEY.md 8(c)'s minimal recipe (oracle/build_ref_sed.sh: only the two
    corona lines, LifeAPI.hpp:1185,1190, made const in a temporary copy; no
    prelude): identical on every fixture input and on fresh seeded batches,
    for every entry point the tests and the bench use."""
    from oracle.oracle import HERE, Ref
    sed = os.path.join(HERE, "_ref", "libref_sed.so")
    if not os.path.exists(sed):
        pytest.skip("oracle/_ref/libref_sed.so not built (make -C oracle ref)")
    a, b = ref, Ref(sed)
    states = [load("random_step.npz")["input"], load("edge_cases.npz")["input"],
              load("randomstate_kat.npz")["input"], load("contains.npz")["states"],
              load("counts.npz")["input"], load("rle.npz")["states"], port.fill(512, seed=808)]
    x = np.concatenate(states)
    for gens in (1, 2, 7, 64):
        assert (a.step_batch(x, gens, nthreads=4) == b.step_batch(x, gens, nthreads=4)).all(), gens
    assert (a.step_alt(x) == b.step_alt(x)).all()
    assert (a.step_nc(x) == b.step_nc(x)).all()
    c = load("contains.npz")
    for w, u in ((c["wanted"], c["unwanted"]), (x[3], x[7] & ~x[3])):
        fa, sa = a.step_contains_batch(x, w, u, 5, nthreads=4)
        fb, sb = b.step_contains_batch(x, w, u, 5, nthreads=4)
        assert (fa == fb).all() and (sa == sb).all()
        assert (a.contains_batch(x, w, u) == b.contains_batch(x, w, u)).all()
        for kind in Ref.PATTERN_KINDS:
            assert (a.pattern_batch(x, kind, w, u, 5, -3) == b.pattern_batch(x, kind, w, u, 5, -3)).all(), kind
    for s in x[:64]:
        assert (a.neighbour_count(s) == b.neighbour_count(s)).all()
        assert (a.interaction_counts(s) == b.interaction_counts(s)).all()
        assert a.rle(s) == b.rle(s) and a.pop(s) == b.pop(s)
        assert all((p == q).all() for p, q in zip(a.target_from_state(s, 3, -9), b.target_from_state(s, 3, -9)))
    r = load("rle.npz")
    for u in range(len(r["parse_offsets"]) - 1):
        t = bytes(r["parse_text"][int(r["parse_offsets"][u]):int(r["parse_offsets"][u + 1])]).decode()
        assert (a.parse(t) == b.parse(t)).all()
    wl = load("weld.npz")["input"]
    assert (a.weld_step(wl, 7) == b.weld_step(wl, 7)).all()
    rf = load("refined_step.npz")["input"]
    assert (a.refined_step(rf) == b.refined_step(rf)).all()
    st = load("stable.npz")["input"]
    for which in range(6):
        pa, pb = st.copy(), st.copy()
        for u in range(len(st)):
            fa_ = a.stable_pass(pa[u], which)
            fb_ = b.stable_pass(pb[u], which)
            assert fa_ == fb_
        assert (pa == pb).all(), which
    for u in range(len(st)):
        assert (a.stable_vulnerable(st[u]) == b.stable_vulnerable(st[u])).all()


def test_filter_iter_digests_from_the_port(port, meta):
    """bench.py secondary_filter_iter's digests (the reference's own Step() +
    Contains loop, make_golden.py filter_iter_digests) reproduced by the
    restatement: first-hit generations of every target at every generation
    count on the full 1M config-2 input"""
    d = meta["digests"]["config2_filter_iter"]
    x = port.fill(d["universes"], d["seed"])
    for name, t in d["targets"].items():
        w, u = (np.array([int(v, 16) for v in t[k]], dtype=np.uint64) for k in ("wanted", "unwanted"))
        care = w | u
        gens = sorted(int(g) for g in t["gens"])
        first, s = np.zeros(len(x), np.uint32), x
        for g in range(1, gens[-1] + 1):
            s = port.step_batch(s, 1, nthreads=8)
            hit = (((s ^ w) & care) == 0).all(axis=1)
            first[(first == 0) & hit] = g
            if str(g) in t["gens"]:
                got = np.where(first <= g, first, 0).astype(np.uint64)
                want = t["gens"][str(g)]
                assert int((got > 0).sum()) == want["hits"], (name, g)
                assert f"{port.digest(got):016x}" == want["first_digest"], (name, g)


def test_stable_window_fixture(port):
    """tests/golden/stable_window.npz (LifeStables on which Propagate's
    window width matters, with the reference's answers): the restatement's
    Propagate agrees"""
    g = load("stable_window.npz")
    got, fl = port.stable_pass(g["input"], 4)
    assert (got == g["propagate"]).all() and (fl == g["flags"]).all()
