"""List VMEM stores whose address or data VGPRs are the destination of an
asynchronous return (ds_read*, buffer_load*, global_load*) issued within the
next N instructions, per kernel of a gfx950 assembly file.  A diagnostic for
the dense-E K5 corruption: the returning write can land
before the store has read its VGPRs.

    python tools/scan_store_war.py file.s [N]
"""
import re
import sys


def regs(tok):
    tok = tok.strip()
    m = re.match(r"v\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def main():
    path = sys.argv[1]
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    kern = None
    lines = open(path).read().splitlines()
    hits = {}
    for n, l in enumerate(lines):
        mk = re.match(r"^(_Z\w+):", l)
        if mk:
            kern = mk.group(1)
        t = l.strip()
        if not (t.startswith("buffer_store") or t.startswith("global_store")):
            continue
        ops = [x for x in t.split(None, 1)[1].split(",")]
        if t.startswith("global_store"):
            src = regs(ops[0]) | regs(ops[1])
        else:
            src = regs(ops[0]) | regs(ops[1])
        for m in range(n + 1, min(n + 1 + N, len(lines))):
            u = lines[m].strip()
            if not u or u.startswith(";") or u.startswith("."):
                continue
            op = u.split(None, 1)
            if len(op) < 2:
                continue
            if op[0].startswith(("ds_read", "buffer_load", "global_load", "ds_bpermute", "ds_swizzle")):
                if regs(op[1].split(",")[0]) & src:
                    hits.setdefault(kern, []).append((n, m - n, op[0], t[:70]))
                    break
    for k, v in hits.items():
        print(k, len(v))
        for h in v[:6]:
            print("   ", h)


if __name__ == "__main__":
    main()
