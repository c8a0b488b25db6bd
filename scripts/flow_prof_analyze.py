"""Analyse per-row timestamps of the sync-free VADU solves (GPBOOST_AMD_FLOW_PROF dumps)."""
import sys

import numpy as np

for fn in sys.argv[1:]:
    raw = open(fn, "rb").read()
    hdr = np.frombuffer(raw, np.int32, 4)
    n, nlev_b, nlev, t = map(int, hdr)
    off = 16
    lptr = np.frombuffer(raw, np.int32, nlev + 1, off); off += 4 * (nlev + 1)
    crit = np.frombuffer(raw, np.int32, 2 * n, off); off += 8 * n
    lrows = np.frombuffer(raw, np.int32, 2 * n, off); off += 8 * n
    prof = np.frombuffer(raw, np.uint64, 8 * n, off).reshape(2 * n, 4).astype(np.int64)
    print(f"== {fn}: n={n} t={t} levels b={nlev_b} total={nlev}")
    for solve, (p0, l0, l1) in enumerate([(0, 0, nlev_b), (n, nlev_b, nlev)]):
        P = prof[p0:p0 + n]
        t0 = P[:, 0][P[:, 0] > 0].min()
        setup, seen, pub = (P[:, 0] - t0) * 10, (P[:, 1] - t0) * 10, (P[:, 2] - t0) * 10   # ns
        pos = np.empty(n, np.int64)
        pos[lrows[p0:p0 + n]] = np.arange(n)
        cr = crit[p0:p0 + n]
        has = cr >= 0
        dep_pub = np.where(has, pub[pos[np.where(has, cr, 0)]], 0)
        lat_seen = (seen - dep_pub)[has & (P[:, 1] > 0)]
        lat_pub = (pub - np.maximum(seen, setup))[has & (P[:, 1] > 0)]
        wait_setup = (setup - dep_pub)[has]
        lev_end = [pub[lptr[l] - p0:lptr[l + 1] - p0].max() for l in range(l0, l1)]
        print(f" solve {solve}: span {pub.max() / 1e3:.1f} us over {l1 - l0} levels "
              f"({pub.max() / 1e3 / (l1 - l0):.2f} us/level)")
        for name, a in [("dep publish -> seen", lat_seen), ("seen -> own publish", lat_pub),
                        ("setup - dep publish (>0: row started late)", wait_setup)]:
            q = np.percentile(a, [10, 50, 90, 99]) / 1e3
            print(f"   {name:45s} p10 {q[0]:7.2f}  p50 {q[1]:7.2f}  p90 {q[2]:7.2f}  p99 {q[3]:7.2f} us")
        le = np.array(lev_end) / 1e3
        d = np.diff(le)
        print(f"   level end times: first 5 {np.round(le[:5], 2)}  median level gap {np.median(d):.2f} us")
