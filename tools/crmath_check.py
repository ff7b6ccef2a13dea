"""Decides tools/crmath_check.cpp's disagreements with mpmath at 200 bits: for each line
"kind a b ours glibc" prints which side is the correctly rounded value. Usage:
    python3 tools/crmath_check.py < disagreements.txt [max_lines]"""
import sys

import mpmath as mp

mp.mp.prec = 200


def rn(v):
    # correctly rounded double of an mpf (mpmath rounds to nearest-even on conversion at 53 bits)
    return float(mp.mpf(v))


def main():
    lim = int(sys.argv[1]) if len(sys.argv) > 1 else 10 ** 9
    cnt = {}
    for i, line in enumerate(sys.stdin):
        if i >= lim:
            break
        k, a, b, ours, gl = line.split()
        a, b, ours, gl = (float.fromhex(t) for t in (a, b, ours, gl))
        if k == "sin":
            t = mp.sin(mp.mpf(a))
        elif k == "cos":
            t = mp.cos(mp.mpf(a))
        else:
            t = mp.atan2(mp.mpf(a), mp.mpf(b))
        cr = rn(t)
        who = "ours" if cr == ours else "glibc" if cr == gl else "neither"
        cnt[(k, who)] = cnt.get((k, who), 0) + 1
        if who != "ours":
            print("NOT CR:", line.strip(), "cr", cr.hex())
    for k, v in sorted(cnt.items()):
        print(k, v)


if __name__ == "__main__":
    main()
