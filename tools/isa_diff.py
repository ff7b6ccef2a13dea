"""Compare the gfx950 machine code of every kernel in two `make asm` outputs (a
refactor of the kernel source must leave the default build's instructions unchanged).

Usage: python tools/isa_diff.py old.s new.s  -> one line per kernel: same / DIFFERENT / only-in-X.
Function-local label numbers and comments are normalised away; metadata is ignored."""
import re
import sys


def kernels(path):
    out, cur, body = {}, None, []
    for ln in open(path):
        m = re.match(r"^(_Z\w+):\s*(;.*)?$", ln)
        if m and not ln.startswith("\t"):
            cur, body = m.group(1), []
            continue
        if cur is None:
            continue
        if re.match(r"^\.Lfunc_end\d+:", ln):
            out[cur] = body
            cur = None
            continue
        t = ln.split(";")[0].rstrip()
        if not t.strip():
            continue
        t = re.sub(r"\.LBB\d+_(\d+)", r".LBB_\1", t)
        t = re.sub(r"\.Ltmp\d+", ".Ltmp", t)
        out.setdefault(cur, None)
        body.append(t)
    return out


def main(a, b):
    ka, kb = kernels(a), kernels(b)
    bad = 0
    for k in sorted(set(ka) | set(kb)):
        if k not in kb:
            print("only-in-old", k)
        elif k not in ka:
            print("only-in-new", k)
            bad += 1
        elif ka[k] == kb[k]:
            print("same", len(ka[k] or []), k)
        else:
            n = sum(1 for x, y in zip(ka[k], kb[k]) if x != y) + abs(len(ka[k]) - len(kb[k]))
            print("DIFFERENT", len(ka[k]), len(kb[k]), n, k)
            bad += 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2]))
