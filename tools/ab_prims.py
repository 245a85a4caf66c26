"""Interleaved A/B of bench.py's primitive timings across libtritd builds.

    python3 tools/ab_prims.py ab/a.so ab/b.so [reps]

Each library is loaded in its own child process (TRITD_LIB), `reps` rounds
alternate between them; prints per-library medians of every primitive's ms.
"""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = (
    "import sys, json; sys.path.insert(0, %r); import bench; "
    "print(json.dumps({k: v['ms'] for k, v in bench.primitives(0, reps=20).items() "
    "if isinstance(v, dict)}))" % ROOT
)


def main():
    libs = [a for a in sys.argv[1:] if a.endswith(".so")]
    reps = int(next((a for a in sys.argv[1:] if a.isdigit()), "4"))
    res = {l: [] for l in libs}
    for k in range(reps):
        for l in libs:
            env = dict(os.environ, TRITD_LIB=os.path.abspath(l))
            out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True,
                                 text=True, timeout=300, cwd=ROOT)
            if out.returncode != 0:
                print(out.stderr[-2000:], flush=True)
                sys.exit(out.returncode)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            res[l].append(d)
            print(k, os.path.basename(l), json.dumps({n: round(v, 4) for n, v in d.items()}),
                  flush=True)
    for l in libs:
        med = {n: round(statistics.median(d[n] for d in res[l]), 4) for n in res[l][0]}
        print("median", os.path.basename(l), json.dumps(med), flush=True)


if __name__ == "__main__":
    main()
