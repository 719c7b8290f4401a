"""Checks tools/fmul_alt_bench's printed sol_mul lines ("sol_mul x[8] y[8] z[8]",
little-endian 32-bit words) with Python integers: z == x y (mod p) and
z < 2^256 (the lazy output; a product chain can take it as input).

    ./tools/fmul_alt_bench | python tools/fmul_alt_check.py
"""
import sys

P = 2**256 - 2**224 + 2**192 + 2**96 - 1


def words(ws):
    return sum(int(w, 16) << (32 * i) for i, w in enumerate(ws))


bad = n = 0
for line in sys.stdin:
    sys.stdout.write(line)
    if not line.startswith("sol_mul"):
        continue
    f = line.split()[1:]
    x, y, z = words(f[0:8]), words(f[8:16]), words(f[16:24])
    n += 1
    if z % P != x * y % P:
        bad += 1
print(f"sol_mul big-integer check: {n - bad} of {n} right")
sys.exit(1 if bad or n == 0 else 0)
