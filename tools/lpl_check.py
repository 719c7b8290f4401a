"""Checks tools/lpl_probe's JSON line against python integers: the chained
products equal x0 y^n 2^(-261 n) mod p, and the chained row-layout XYZZ
additions equal the same add-2008-s sequence mod p (every row's copy).
Measurement tool."""
import json
import sys

P = 2**256 - 2**224 + 2**192 + 2**96 - 1
RI = pow(2**261, -1, P)


def val(limbs):
    return sum(int(v) << (29 * i) for i, v in enumerate(limbs))


def mm(a, b):
    return a * b * RI % P


d = json.loads(sys.stdin.readline())
x0, y = val(d["x0"]), val(d["y"])
ok = True
for k in ("lane", "row", "row2"):
    n = d[k]["iters"] if k != "row2" else d[k]["iters"] // 2
    want = x0 * pow(y, n, P) * pow(RI, n, P) % P
    got = val(d[k]["out"]) % P
    good = got == want and (k != "row2" or val(d[k]["out2"]) % P == want)
    ok &= good
    print(k, d[k]["cycles_per_op"], "cycles", d[k]["ns_per_op"], "ns per product", "OK" if good else "WRONG")
pts = d["pts"]
A = [val(pts[9 * k:9 * k + 9]) for k in range(4)]
B = [val(pts[36 + 9 * k:36 + 9 * k + 9]) for k in range(4)]
for _ in range(d["add"]["iters"]):
    U1, U2, S1, S2 = mm(A[0], B[2]), mm(B[0], A[2]), mm(A[1], B[3]), mm(B[1], A[3])
    Pp, R = (U2 - U1) % P, (S2 - S1) % P
    PP, RR, Z12, ZZZ12 = mm(Pp, Pp), mm(R, R), mm(A[2], B[2]), mm(A[3], B[3])
    PPP, Q, ZZ3 = mm(Pp, PP), mm(U1, PP), mm(Z12, PP)
    X3 = (RR - PPP - 2 * Q) % P
    A = [X3, (mm(R, Q - X3) - mm(S1, PPP)) % P, ZZ3, mm(ZZZ12, PPP)]
out = d["add"]["out"]
good = all(val(out[36 * k + 9 * r:36 * k + 9 * r + 9]) % P == A[k] for k in range(4) for r in range(4))
ok &= good
print("add", d["add"]["cycles_per_op"], "cycles", d["add"]["ns_per_op"], "ns per XYZZ addition", "OK" if good else "WRONG")
sys.exit(0 if ok else 1)
