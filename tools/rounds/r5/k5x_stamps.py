"""Summarise the K5X_STAMPS diagnosis build's per-workgroup stamps
(s_memrealtime, 100 MHz) of one k5_f32s launch: prologue / walk / epilogue
shares and how full each CU's two workgroup slots were.
usage: python tools/rounds/r5/k5x_stamps.py stamps.bin"""
import sys
import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8).astype(np.int64)
t0, t1, t2, t3 = (a[:, q] for q in range(4))
hw, xcc = a[:, 4], a[:, 5] & 0xF
ok = (t0 > 0) & (t3 >= t0)
t0, t1, t2, t3, hw, xcc = t0[ok], t1[ok], t2[ok], t3[ok], hw[ok], xcc[ok]
ns = 10.0
span = (t3.max() - t0.min()) * ns / 1e3
pro, walk, epi, life = (t1 - t0) * ns, (t2 - t1) * ns, (t3 - t2) * ns, (t3 - t0) * ns
print(f"workgroups {len(t0)}  launch span {span:.1f} us (first start -> last end)")
for name, v in (("prologue", pro), ("walk", walk), ("epilogue", epi), ("lifetime", life)):
    print(f"  {name:9s} median {np.median(v)/1e3:7.2f} us  p10 {np.percentile(v,10)/1e3:7.2f}  p90 {np.percentile(v,90)/1e3:7.2f}  share {v.sum()/life.sum():.3f}")
cu = (xcc << 16) | (((hw >> 13) & 0x7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF)
ucu = np.unique(cu)
print(f"CUs seen {len(ucu)}; workgroups per CU median {np.median(np.bincount(np.searchsorted(ucu, cu))):.0f}")
# slot fill: per CU, busy workgroup-time / (2 slots x the CU's own first-start..last-end)
fill, gaps = [], []
for c in ucu:
    m = cu == c
    s0, s3 = np.sort(t0[m]), np.sort(t3[m])
    fill.append((t3[m] - t0[m]).sum() / (2.0 * (s3[-1] - s0[0])))
    # start of each workgroup after the first two vs the end that freed its slot
    if len(s0) > 2:
        gaps.append(np.median((s0[2:] - s3[:len(s0) - 2]) * ns))
print(f"slot fill (2 per CU) median {np.median(fill):.3f}  min {np.min(fill):.3f}")
print(f"slot turnover (next start - freeing end) median over CUs {np.median(gaps)/1e3:.2f} us")
print(f"ramp: 10% of workgroups started by {(np.percentile(t0,10)-t0.min())*ns/1e3:.1f} us, last start at {(t0.max()-t0.min())*ns/1e3:.1f} us; tail after last start {(t3.max()-t0.max())*ns/1e3:.1f} us")
