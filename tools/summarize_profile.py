"""Condense a tools/profile_round.sh output directory into profiles/<tag>_*.

usage: python tools/summarize_profile.py gpurun_out/prof_r01 r01
Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, names shortened) and
profiles/<tag>_hbm_traffic.csv (per-kernel mean FETCH_SIZE / WRITE_SIZE per
dispatch in KB as reported, plus bytes with the gfx950 FETCH_SIZE x2 correction
of MI355X_MICROARCH.md section HBM), profiles/<tag>_build.json (the source hash of
the library the counters were collected on: bench.py reports roofline.traffic only
from a summary of the same sources), and profiles/<tag>_mfma_util.csv, per kernel:
  mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (dur x SCLK x 1024 SIMDs): the busy
      cycles over the kernel's own duration -- the mean duration of the same kernel
      in the counter-free kernel-trace pass (the counter pass serialises and slows
      dispatches) -- at the shader clock measured on the long dispatches of the
      same pass (sclk_ghz: GRBM_GUI_ACTIVE per XCD over the duration of the
      dispatches >= 1 ms, median). (The GRBM-per-XCD form of the rocprofv3 derived
      counter implied 2.4-12.8 GHz clocks for sub-100 us dispatches, VERDICT r03 item
      7 / r04 item 7: not written.)
"""
import json
import os
import re
import sys

import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import source_sha  # noqa: E402


def short(n):
    n = re.sub(r"\(.*", "", n)
    return n if len(n) < 60 else n[:57] + "..."


def main(d, tag, pre="bench"):
    os.makedirs("profiles", exist_ok=True)
    s = pd.read_csv(os.path.join(d, "trace", f"{pre}_kernel_stats.csv"))
    s["Name"] = s["Name"].map(short)
    s = s[["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]]
    s.to_csv(f"profiles/{tag}_kernel_stats.csv", index=False)
    rows = []
    for kind, cname in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        p = os.path.join(d, kind, f"{pre}_counter_collection.csv")
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
    p = os.path.join(d, "mfma", f"{pre}_counter_collection.csv")
    if os.path.exists(p):
        c = pd.read_csv(p)
        c["Name"] = c["Kernel_Name"].map(short)
        g = c.groupby(["Name", "Dispatch_Id", "Counter_Name"]).Counter_Value.sum().unstack().reset_index()
        tr = pd.read_csv(os.path.join(d, "mfma", f"{pre}_kernel_trace.csv"))
        tr["dur_ns"] = tr.End_Timestamp - tr.Start_Timestamp
        g = g.merge(tr[["Dispatch_Id", "dur_ns"]], on="Dispatch_Id")
        g["grbm_per_xcd"] = g.GRBM_GUI_ACTIVE / 8
        g["clock_ghz"] = g.grbm_per_xcd / g.dur_ns
        long_ = g[g.dur_ns >= 1e6]
        sclk = float(long_.clock_ghz.median()) if len(long_) else 2.0
        m = g.groupby("Name")[["SQ_VALU_MFMA_BUSY_CYCLES", "dur_ns"]].median()
        m = m.reset_index()
        # the kernel's own duration: the counter-free trace pass's mean (ns)
        trace_mean = dict(zip(s["Name"], s["AverageNs"]))
        m["trace_dur_ns"] = m["Name"].map(trace_mean)
        m["sclk_ghz"] = sclk
        m["mfma_util"] = m.SQ_VALU_MFMA_BUSY_CYCLES / (m.trace_dur_ns.fillna(m.dur_ns) * sclk * 1024)
        # over every dispatch of the kernel (sizes vary within a factor): summed busy
        # cycles over summed durations of the same counter pass
        tot = g.groupby("Name")[["SQ_VALU_MFMA_BUSY_CYCLES", "dur_ns"]].sum()
        m["mfma_util_all_dispatches"] = m["Name"].map(tot.SQ_VALU_MFMA_BUSY_CYCLES / (tot.dur_ns * sclk * 1024))
        m.to_csv(f"profiles/{tag}_mfma_util.csv", index=False)
        print(m.to_string())
    with open(f"profiles/{tag}_build.json", "w") as f:
        json.dump({"tag": tag, "src_sha": source_sha(), "profile_dir": d}, f)
    print(s.head(8).to_string())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(sys.argv[3:4]))
