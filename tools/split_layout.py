"""Check the row-split layout tables of csrc/split_layout.hpp (SplitNet<S>): the
five index-bit swaps map universe u, row S*k + j to register j, bit P*k + u,
and running them backwards restores the columns.  Pure Python, no GPU."""
import random
import re
import sys

M = 0xFFFFFFFF
MASKS = [0x0000FFFF, 0x00FF00FF, 0x0F0F0F0F, 0x33333333, 0x55555555]


def tables(src):
    out = {}
    for s, body in re.findall(r"struct SplitNet<(\d+)> \{.*?\n(.*?)\n\};", src, re.S):
        a = [int(v) for v in re.search(r"a\[5\] = \{([^}]*)\}", body)[1].split(",")]
        expr = re.search(r"reg\(int j\) \{ return (.*?); \}", body)[1]
        out[int(s)] = (a, eval("lambda j: " + expr))
    return out


def swap(x, a, stage):
    x = list(x)
    sh, m = 16 >> stage, MASKS[stage]
    for i in range(len(x)):
        if not (i >> a) & 1:
            k = i | (1 << a)
            t = ((x[i] >> sh) ^ x[k]) & m
            x[k] ^= t
            x[i] = (x[i] ^ (t << sh)) & M
    return x


def check(src):
    for S, (a, reg) in tables(src).items():
        P = S // 2
        for _ in range(50):
            cols = [random.getrandbits(64) for _ in range(P)]
            x = [w for c in cols for w in (c & M, c >> 32)]
            for st in range(5):
                x = swap(x, a[st], st)
            r = [x[reg(j)] for j in range(S)]
            for j in range(S):
                for k in range(64 // S):
                    for u in range(P):
                        assert (r[j] >> (P * k + u)) & 1 == (cols[u] >> (S * k + j)) & 1, (S, j, k, u)
            y = [0] * S
            for j in range(S):
                y[reg(j)] = r[j]
            for st in reversed(range(5)):
                y = swap(y, a[st], st)
            assert [y[2 * u] | (y[2 * u + 1] << 32) for u in range(P)] == cols
    return sorted(tables(src))


if __name__ == "__main__":
    print("ok", check(open(sys.argv[1] if len(sys.argv) > 1 else "lifeapi_amd/csrc/split_layout.hpp").read()))
