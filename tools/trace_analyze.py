"""Offline analysis of tools/trace_dump.py output (argv[1], .npz): the lattice step's
chain per GP and per XCD. Role layout of launch 1 (per GP, GP fastest): the P scan
units, nprod producers, nwu w units, nzu Z units; k_lat_gemm2 at 1024 + tile.
Slots: w units 0 start / 1 past the L21 wait / 3 F loop done / 2 published (last
arrivers); Z units 0 start / 1 lists read / 3 past the w wait / 2 published; GEMM 0 start /
2 K loop done / 3 splits met / 6 cells done / 4 end."""
import sys
import numpy as np

d = np.load(sys.argv[1])
raw_all = d["raw"]
B = int(d["B"])
NPROD, NWU, NZU, P = int(sys.argv[2]) if len(sys.argv) > 2 else 16, 64, 64, 2
q = lambda a: " ".join(f"{np.nanpercentile(a, p):6.1f}" for p in (0, 10, 50, 90, 100)) if np.isfinite(a).any() else "-"
for rep, raw in enumerate(raw_all):
    NWG = raw.shape[0]
    tr = raw[:, :7].astype(np.float64)
    used = tr[:, 0] > 0
    t0 = tr[used, 0].min()
    tr = np.where(tr > 0, (tr - t0) / 100.0, np.nan)
    lin = np.arange(NWG)
    gp = lin % B
    role = lin // B
    hw = raw[:, 7]
    xcc = (hw >> 32) & 0xF
    cu = xcc * 1024 + ((hw >> 13) & 0x7) * 64 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 0xF)
    r1 = role - P
    isw = (r1 >= NPROD) & (r1 < NPROD + NWU) & used
    isz = (r1 >= NPROD + NWU) & (r1 < NPROD + NWU + NZU) & used
    isp = (r1 >= 0) & (r1 < NPROD) & used
    isg = (role >= 1024) & used
    print(f"--- step {rep}: last WG end {np.nanmax(tr):.1f} us")
    print(f"  producers done (slot 1): {q(tr[isp, 1])}")
    print(f"  w past L21 wait: {q(tr[isw, 1])}")
    print(f"  w F loop end   : {q(tr[isw, 3])}")
    print(f"  w F loop length: {q(tr[isw, 3] - tr[isw, 1])}")
    print(f"  w published    : {q(tr[isw, 2])}")
    print(f"  Z past w wait  : {q(tr[isz, 3])}")
    print(f"  Z published    : {q(tr[isz, 2])}")
    g0 = tr[isg, 0]
    print(f"  gemm start     : {q(g0)}")
    print(f"  gemm Z built   : {q(tr[isg, 1])}  (lat_zl2)")
    print(f"  gemm Z waited  : {q(tr[isg, 5])}  (lat_zl2)")
    print(f"  gemm K done    : {q(tr[isg, 2])}  (K loop {q(tr[isg, 2] - tr[isg, 0])})")
    print(f"  gemm end       : {q(tr[isg, 4])}")
    print("  per GP: [w F-loop end max, w publ max, Z publ max] ; per XCC of its w units")
    for g in range(B):
        sw, sz = isw & (gp == g), isz & (gp == g)
        xs = np.unique(xcc[sw])
        mx = lambda a: np.nanmax(a) if np.isfinite(a).any() else float("nan")
        print(f"    GP {g}: {mx(tr[sw, 3]):6.1f} {mx(tr[sw, 2]):6.1f} {mx(tr[sz, 2]):6.1f}   xcc {xs}")
    print("  per XCC: w F-loop length p50/max, #w units, #CUs used by w")
    for x in range(8):
        sw = isw & (xcc == x)
        if sw.any():
            ln = tr[sw, 3] - tr[sw, 1]
            print(f"    XCC {x}: {np.nanmedian(ln):6.1f} {np.nanmax(ln):6.1f}  n={sw.sum():3d} cus={len(np.unique(cu[sw]))}")
    # per CU: units on it and the later one's F loop end
    wcu = cu[isw]
    ends = tr[isw, 3]
    starts = tr[isw, 0]
    order = {}
    for c, s, e in zip(wcu, starts, ends):
        order.setdefault(c, []).append((s, e))
    firsts, seconds = [], []
    for c, lst in order.items():
        lst.sort()
        firsts.append(lst[0][1])
        if len(lst) > 1:
            seconds.append(lst[1][1])
    print(f"  CU's first-dispatched w unit ends: {q(np.array(firsts))}; second: {q(np.array(seconds))}")
    hist = np.bincount([len(v) for v in order.values()])
    print(f"  w units per CU histogram: {dict(enumerate(hist))}")
    # other roles sharing a CU with the last-finishing w units
    late = np.argsort(-np.nan_to_num(tr[:, 3] * isw, nan=-1))[:10]
    for i in late:
        c = cu[i]
        share = [(int(role[j] - P), int(gp[j])) for j in np.nonzero((cu == c) & used & (role < 1024))[0] if j != i]
        print(f"    late w: GP {gp[i]} unit {r1[i] - NPROD} xcc {xcc[i]} start {tr[i,0]:.1f} L21 {tr[i,1]:.1f} end {tr[i,3]:.1f}; CU shared with roles {share}")
