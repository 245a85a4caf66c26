"""Wide-store data rewrite scanner for gfx950 code objects.

Lists every wide VMEM store (more than 64 bits of data per lane:
`buffer_store_dwordx3/x4`, `global_store_dwordx3/x4`) whose data VGPRs a
VALU or MFMA instruction rewrites within the next N issued instructions, on
any control path that leaves the store (`s_nop k` counts as k + 1; with
--all, asynchronous returns — `ds_read*`, `*_load_*` — are listed too).

Why (profiles/round5/store_hazard_probe.txt): on MI355X a
VALU write of a wide store's data registers with no wait state after the
store replaces the data of lanes 12-15 of each 16 (the 64-bit word it
writes).  The ISA asks for one wait state there, and LLVM's hazard
recognizer inserts it — except for MUBUF stores that take an SGPR soffset,
which it treats as hazard-free.  K5 streams Y_L, E and T through exactly
such stores (wave-uniform buffer descriptors, the t-tile offset in an
SGPR), and a build of K5 without its store-data keeps
(`-DTRITD_STORE_KEEP=0`) has the compiler put `v_add_f64` /
`v_lshl_add_u64` / `v_fma_f64` writes of the data pair right behind such
stores: the round-4 dense-E corruption, which that build reproduces on the
GPU (profiles/round5/nokeep_determinism.txt).  With a constant soffset one
wait state was not always enough in the probe either (16 of 67M lanes
wrong), so the check asks for two: a synchronous rewrite at distance <= 2.

`tests/test_isa_store_war.py` runs it over every code object of the shipped
libtritd.so (none allowed) and over a K5 built without the keeps (caught).

    python tools/scan_store_war.py [--all] [N] [lib.so | object.o ...]
        (default: N = WINDOW, the in-tree libtritd.so)
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
# a synchronous rewrite of wide-store data at this distance or less (issued
# instructions from the store; 1 = the next one) is reported: at least two
# wait states are required (module docstring)
WINDOW = 2
HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "triple-tensor-decomposition-with-admm_amd", "csrc")

_INS = re.compile(r"^\s+([a-z_0-9]+)(\s+(.*?))?\s*//\s*([0-9A-Fa-f]+):")
_FUN = re.compile(r"^[0-9a-f]+ <([^>]+)>:")
_WIDE = re.compile(r"^(buffer|global|flat)_store_dwordx[34]$")
_BR = re.compile(r"^s_(c?branch\w*)$")


def vregs(tok):
    """VGPR numbers named by one operand (v5, v[4:7]); AGPRs are not VGPRs."""
    tok = tok.strip()
    m = re.match(r"v\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def split_ops(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def parse(dis):
    """{function: [(addr, mnemonic, operands)]} from llvm-objdump -d text."""
    funs, cur = {}, None
    for line in dis.splitlines():
        m = _FUN.match(line)
        if m:
            cur = funs.setdefault(m.group(1), [])
            continue
        m = _INS.match(line)
        if m and cur is not None:
            cur.append((int(m.group(4), 16), m.group(1), split_ops(m.group(3) or "")))
    return funs


def writes_vgprs(mn, ops):
    """VGPRs an instruction writes (its first operand), or none."""
    if not ops:
        return set()
    if mn.startswith(("s_", "buffer_store", "global_store", "flat_store", "scratch_store",
                      "ds_write", "ds_store", "exp")):
        return set()
    if mn.startswith(("v_", "ds_", "buffer_", "global_", "flat_", "scratch_")):
        if mn.startswith(("v_readlane", "v_readfirstlane", "v_cmp")):
            return set()
        if mn.startswith(("buffer_atomic", "global_atomic", "flat_atomic")) and "glc" not in " ".join(ops) \
                and "sc0" not in " ".join(ops):
            return set()
        return vregs(ops[0])
    return set()


def branch_target(mn, ops, addr):
    # objdump prints the target as a byte offset from the next instruction
    # (s_branch 65517 // ...) or as an absolute label; both forms handled
    if not ops:
        return None
    t = ops[0].split()[0]
    try:
        v = int(t, 0)
    except ValueError:
        return None
    if v >= 32768:
        v -= 65536
    return addr + 4 + 4 * v


def is_async(mn):
    """Writers whose register write comes back later through a memory return
    path (LDS or VMEM loads), not in the VALU pipeline."""
    return mn.startswith(("ds_", "buffer_", "global_", "flat_", "scratch_"))


def scan_function(ins, window=WINDOW, sync_only=False):
    """[(store_addr, store_text, distance, writer_text)] inside the window.
    distance: issued instructions from the store to the writer (1 = the next
    one, no wait state between them).  sync_only: VALU / MFMA writers only."""
    index = {a: n for n, (a, _, _) in enumerate(ins)}
    hits = []
    for n, (addr, mn, ops) in enumerate(ins):
        if not _WIDE.match(mn):
            continue
        data = vregs(ops[1] if mn.startswith(("global", "flat")) else ops[0])
        if not data:
            continue
        # breadth over paths: (instruction index, issued count so far)
        todo, seen, found = [(n + 1, 0)], set(), None
        while todo and found is None:
            k, cnt = todo.pop()
            while k < len(ins) and cnt < window:
                if (k, cnt) in seen:
                    break
                seen.add((k, cnt))
                a2, m2, o2 = ins[k]
                cnt += (int(o2[0], 0) + 1) if (m2 == "s_nop" and o2) else 1
                if writes_vgprs(m2, o2) & data and cnt <= window and not (sync_only and is_async(m2)):
                    found = (cnt, m2 + " " + ", ".join(o2))
                    break
                if m2 in ("s_endpgm", "s_setpc_b64"):
                    break
                mb = _BR.match(m2)
                if mb:
                    tgt = branch_target(m2, o2, a2)
                    if tgt in index:
                        todo.append((index[tgt], cnt))
                    if m2 == "s_branch":
                        break
                k += 1
        if found:
            hits.append((addr, mn + " " + ", ".join(ops), found[0], found[1]))
    return hits


def code_objects(path):
    """The gfx950 code objects inside a built .o or the linked .so: its
    .hip_fatbin section holds one offload bundle per translation unit."""
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", path,
                        os.path.join(td, "x")], check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), data)]
        out = []
        for n, a in enumerate(starts):
            b = starts[n + 1] if n + 1 < len(starts) else len(data)
            part, co = os.path.join(td, f"b{n}"), os.path.join(td, f"co{n}")
            open(part, "wb").write(data[a:b])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}",
                            f"--output={co}", "--unbundle"], check=True, capture_output=True)
            out.append(open(co, "rb").read())
        return out


def disassemble(blob):
    with tempfile.TemporaryDirectory() as td:
        co = os.path.join(td, "co")
        open(co, "wb").write(blob)
        r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                           capture_output=True, text=True)
        return r.stdout


def scan_object(path, window=WINDOW, sync_only=False):
    """{function: hits} over every code object of a built .o or .so."""
    out = {}
    for blob in code_objects(path):
        for f, ins in parse(disassemble(blob)).items():
            h = scan_function(ins, window, sync_only)
            if h:
                out[f] = h
    return out


def has_device_code(path):
    r = subprocess.run([f"{LLVM}/llvm-readelf", "-S", path], capture_output=True, text=True)
    return ".hip_fatbin" in r.stdout


def main():
    args = sys.argv[1:]
    sync_only = True
    if args and args[0] == "--all":
        sync_only = False
        args.pop(0)
    window = WINDOW
    if args and args[0].isdigit():
        window = int(args.pop(0))
    objs = args or [os.path.join(CSRC, "..", "tritd", "libtritd.so")]
    total = 0
    for o in objs:
        if not has_device_code(o):
            continue
        for f, hs in scan_object(o, window, sync_only).items():
            print(f"{os.path.basename(o)} {f}: {len(hs)}")
            for h in hs:
                print(f"    0x{h[0]:x} {h[1][:60]:60s} +{h[2]:2d} {h[3][:60]}")
            total += len(hs)
    print(f"{total} wide-store data rewrites within {window} instructions")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
