"""List wide VMEM stores (dwordx3/x4: more than 64 bits of data per lane)
whose data VGPRs are rewritten within the next N instructions — by a VALU
instruction or by an asynchronous return (ds_read*, buffer_load*,
global_load*) — per kernel of a gfx950 assembly file.

On MI355X such a rewrite 3-4 instructions after a `buffer_store_dwordx4`
(the compiler's hazard padding is satisfied) was measured to replace the
store's first 64-bit word in lanes 12-15 of each 16 now and then: the
dense-E K5 corruption of round 4.  The kernels hold the
data of their wide stores live past a later point instead (K5_KEEP).

    python tools/scan_store_war.py file.s [N] [kernel-substring]
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


def scan(lines, N, want=""):
    kern = None
    hits = {}
    for n, l in enumerate(lines):
        mk = re.match(r"^(_Z\w+):", l)
        if mk:
            kern = mk.group(1)
        if want and (kern is None or want not in kern):
            continue
        t = l.strip()
        if not re.match(r"(buffer|global)_store_dwordx[34]\b", t):
            continue
        ops = t.split(None, 1)[1].split(",")
        data = regs(ops[1]) if t.startswith("global_store") else regs(ops[0])
        cnt = 0
        for m in range(n + 1, len(lines)):
            u = lines[m].strip()
            if not u or u.startswith(";") or u.startswith("."):
                continue
            if u.endswith(":"):  # a label: the path forks
                break
            cnt += 1
            if cnt > N:
                break
            op = u.split(None, 1)
            if len(op) < 2 or "store" in op[0] or op[0].startswith(("ds_write", "s_", "v_mfma")):
                continue
            if regs(op[1].split(",")[0]) & data:
                hits.setdefault(kern, []).append((n + 1, cnt, op[0], t[:64]))
                break
    return hits


def main():
    path = sys.argv[1]
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    want = sys.argv[3] if len(sys.argv) > 3 else ""
    hits = scan(open(path).read().splitlines(), N, want)
    for k, v in hits.items():
        print(k, len(v))
        for h in v:
            print("   ", h)


if __name__ == "__main__":
    main()
