#!/usr/bin/env python3
"""Summarise a KCTC_REC_TRACE recurrence trace (rec_fwd.bin / rec_bwd.bin).

Per phase: median over steps 8..steps-1 and over workgroups of the phase
duration (us, 100 MHz stamps); plus the hand-off latency = consumer
'flags seen' minus the LAST producer's 'published' of the previous step."""
import sys
import numpy as np


def main(path):
    raw = open(path, "rb").read()
    grid, steps, nwg, T, dirs, ver, xpd, stride = np.frombuffer(raw[:32], dtype=np.int32)
    tr = np.frombuffer(raw[32:], dtype=np.uint64).reshape(steps, grid, stride or 16).astype(np.int64)
    steps = min(steps, T)
    tr = tr[:steps]
    if xpd == 0:  # v6: block b -> (dir b % dirs, g b / dirs)
        members = [[b for b in range(grid) if b % dirs == d and b // dirs < nwg] for d in range(dirs)]
    elif ver >= 4:
        members = [[b for b in range(grid) if (b % 8) // xpd == d and (b // 8) * xpd + (b % 8) % xpd < nwg]
                   for d in range(dirs)]
    else:
        members = [list(range(d * nwg, (d + 1) * nwg)) for d in range(dirs)]
    active = sorted(b for m in members for b in m)
    tr = tr[:, active, :]
    loc = tr[0, :, 9]
    if loc.max() > 0 and loc.max() < 8:  # v6 backward: hand-off mode per workgroup (1 sc1, 2 XCD-local)
        print(f"  XCD-local workgroups: {int((loc == 2).sum())} of {len(loc)}")
    idx = {b: i for i, b in enumerate(active)}
    us = 1e-2  # 100 MHz
    names = ["start->flags", "flags->loads", "loads->reduced", "reduced->published", "published->end"]
    sl = slice(8, steps)
    print(f"{path}: v{ver} grid={grid} nwg={nwg} xpd={xpd} dirs={dirs} T={T} steps traced={steps}")
    m = (tr[sl, :, 15] - tr[sl, :, 14]).astype(np.float64)
    r = (tr[sl, :, 3] - tr[sl, :, 2]).astype(np.float64) * 1e-8
    ok = (r > 0) & (m > 0)
    if ok.any():
        print(f"  shader clock (s_memtime / s_memrealtime) ~{np.median(m[ok] / r[ok]) / 1e9:.2f} GHz")
    # phases this kernel records (slot 7: hand-off stores issued, before the drain), in time order
    stamps = [i for i in (0, 1, 2, 8, 12, 3, 7, 4, 5) if tr[sl, :, i].min() > 0]
    stamps.sort(key=lambda i: np.median(tr[sl, :, i] - tr[sl, :, 0]))
    pnames = {0: "start", 1: "flags", 2: "loads", 3: "reduced", 4: "published", 5: "end", 7: "stored",
              8: "barrier1", 12: "cell"}
    for a, b in zip(stamps[:-1], stamps[1:]):
        d = (tr[sl, :, b] - tr[sl, :, a]) * us
        nm = f"{pnames[a]}->{pnames[b]}"
        print(f"  {nm:22s} median {np.median(d):7.3f}  p90 {np.percentile(d, 90):7.3f}")
    if tr.shape[2] >= 32 and tr[sl, :, 16].min() > 0:  # v6 backward: per-wave flags / loads
        nwv = max(w for w in range(8) if tr[sl, :, 16 + w].min() > 0) + 1
        for w in range(nwv):
            fl = (tr[sl, :, 16 + w] - tr[sl, :, 0]) * us
            ld = (tr[sl, :, 24 + w] - tr[sl, :, 0]) * us
            print(f"  wave {w}: start->flags {np.median(fl):7.3f}  start->{'mfma issued' if 'fwd' in path else 'loads'} "
                  f"{np.median(ld):7.3f}")
        last = tr[sl, :, 24:24 + nwv].max(axis=2)
        nxt = 8 if tr[sl, :, 8].min() > 0 else 3
        print(f"  last wave's stamp->{pnames[nxt]} median {np.median((tr[sl, :, nxt] - last) * us):7.3f}"
              f"  start->last wave's stamp {np.median((last - tr[sl, :, 0]) * us):7.3f}")
    elif ver >= 4 and tr[sl, :, 6].min() > 0:
        for w in range(4):
            ld = (tr[sl, :, 6 + w] - tr[sl, :, 1]) * us
            mf = (tr[sl, :, 10 + w] - tr[sl, :, 6 + w]) * us
            print(f"  wave {w}: flags->loads {np.median(ld):7.3f}  loads->mfma-done {np.median(mf):7.3f}")
    step = (tr[9:steps, :, 0] - tr[8:steps - 1, :, 0]) * us
    print(f"  step period            median {np.median(step):7.3f}  p90 {np.percentile(step, 90):7.3f}")
    lat = []
    for d, m in enumerate(members):
        cols = [idx[b] for b in m]
        pub = tr[8:steps - 1][:, cols, 4]
        seen = tr[9:steps][:, cols, 1]
        lat.append((seen - pub.max(axis=1)[:, None]) * us)
        print(f"  dir {d}: publish skew (last-first producer) median {np.median((pub.max(1) - pub.min(1)) * us):.3f}")
    lat = np.concatenate([l.ravel() for l in lat])
    print(f"  handoff last-publish->seen median {np.median(lat):7.3f}  p10 {np.percentile(lat, 10):7.3f}  "
          f"p90 {np.percentile(lat, 90):7.3f}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
