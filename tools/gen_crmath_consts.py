"""Prints the double-double constants of tools/crmath.h (Taylor coefficients (-1)^k / (2k+1)!,
(-1)^k / (2k)!, pi/2 in four parts) from mpmath at 300 bits. Run once; the output is pasted into the
header, so this script documents where those numbers come from."""
import mpmath as mp

mp.mp.prec = 300


def split(v):
    h = float(v)
    return h, float(v - mp.mpf(h))


print("// sin: (-1)^k / (2k+1)!, k = 1..13")
for k in range(1, 14):
    h, l = split(mp.mpf(-1) ** k / mp.factorial(2 * k + 1))
    print(f"    {{{h!r}, {l!r}}},")
print("// cos: (-1)^k / (2k)!, k = 1..14")
for k in range(1, 15):
    h, l = split(mp.mpf(-1) ** k / mp.factorial(2 * k))
    print(f"    {{{h!r}, {l!r}}},")
# pi/2 = P1 + P2 + P3 + P4: P1..P3 carry 33 bits each (n * Pi exact for n < 2^20), P4 53 bits
v = mp.pi / 2
parts = []
for bits in (33, 33, 33):
    e = mp.floor(mp.log(abs(v), 2))
    q = mp.mpf(2) ** (e - bits + 1)
    p = mp.floor(v / q) * q
    parts.append(float(p))
    v -= p
parts.append(float(v))
print("// pi/2 parts:", ", ".join(repr(p) for p in parts))
print("// residual after 4 parts:", float(mp.pi / 2 - sum(mp.mpf(p) for p in parts)))
h, l = split(mp.pi)
print("// pi:", repr(h), repr(l))
