"""Condense a tools/profile_round.sh output directory into profiles/<tag>_*.

usage: python tools/summarize_profile.py gpurun_out/prof_r01 r01
Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, names shortened) and
profiles/<tag>_hbm_traffic.csv (per-kernel mean FETCH_SIZE / WRITE_SIZE per
dispatch in KB as reported, plus bytes with the gfx950 FETCH_SIZE x2 correction
of MI355X_MICROARCH.md section HBM), and profiles/<tag>_mfma_util.csv (per-kernel
MfmaUtil = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE per XCD x 1024 SIMDs), the
rocprofv3 derived-counter formula; the CSV's GRBM_GUI_ACTIVE is the sum over the 8
XCDs, so it is divided by 8, and the clock it implies).
"""
import os
import re
import sys

import pandas as pd


def short(n):
    n = re.sub(r"\(.*", "", n)
    return n if len(n) < 60 else n[:57] + "..."


def main(d, tag):
    os.makedirs("profiles", exist_ok=True)
    s = pd.read_csv(os.path.join(d, "trace", "bench_kernel_stats.csv"))
    s["Name"] = s["Name"].map(short)
    s = s[["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]]
    s.to_csv(f"profiles/{tag}_kernel_stats.csv", index=False)
    rows = []
    for kind, cname in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        p = os.path.join(d, kind, "bench_counter_collection.csv")
        if not os.path.exists(p):
            continue
        c = pd.read_csv(p)
        c["Name"] = c["Kernel_Name"].map(short)
        g = c[c.Counter_Name == cname].groupby("Name")["Counter_Value"].agg(["mean", "count"]).reset_index()
        g["counter"] = cname
        rows.append(g)
    if rows:
        t = pd.concat(rows).pivot_table(index="Name", columns="counter", values="mean").reset_index()
        if "FETCH_SIZE" in t:
            t["fetch_bytes_corrected"] = t["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in t:
            t["write_bytes"] = t["WRITE_SIZE"] * 1024
        t.to_csv(f"profiles/{tag}_hbm_traffic.csv", index=False)
        print(t.to_string())
    p = os.path.join(d, "mfma", "bench_counter_collection.csv")
    if os.path.exists(p):
        c = pd.read_csv(p)
        c["Name"] = c["Kernel_Name"].map(short)
        g = c.groupby(["Name", "Dispatch_Id", "Counter_Name"]).Counter_Value.sum().unstack().reset_index()
        tr = pd.read_csv(os.path.join(d, "mfma", "bench_kernel_trace.csv"))
        tr["dur_ns"] = tr.End_Timestamp - tr.Start_Timestamp
        g = g.merge(tr[["Dispatch_Id", "dur_ns"]], on="Dispatch_Id")
        g["grbm_per_xcd"] = g.GRBM_GUI_ACTIVE / 8
        g["mfma_util"] = g.SQ_VALU_MFMA_BUSY_CYCLES / (g.grbm_per_xcd * 1024)
        g["clock_ghz"] = g.grbm_per_xcd / g.dur_ns
        m = g.groupby("Name")[["mfma_util", "clock_ghz", "SQ_VALU_MFMA_BUSY_CYCLES", "grbm_per_xcd", "dur_ns"]].median()
        m = m.reset_index()
        m.to_csv(f"profiles/{tag}_mfma_util.csv", index=False)
        print(m.to_string())
    print(s.head(8).to_string())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
