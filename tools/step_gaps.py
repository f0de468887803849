"""Per-step timeline of the two-launch lattice step from a rocprofv3 kernel trace:
median durations of k_inc_lat_arg, the gap to k_lat_gemm2_arg, its duration, and
the gap to the next step's first launch (us)."""
import sys

import numpy as np
import pandas as pd

t = pd.read_csv(sys.argv[1]).sort_values("Start_Timestamp")
names, st, en = t["Kernel_Name"].tolist(), t["Start_Timestamp"].to_numpy(), t["End_Timestamp"].to_numpy()
seq = [(en[i] - st[i], st[i + 1] - en[i], en[i + 1] - st[i + 1], st[i + 2] - en[i + 1], st[i + 2] - st[i])
       for i in range(len(names) - 2)
       if "k_inc_lat_arg" in names[i] and "k_lat_gemm2_arg" in names[i + 1] and "k_inc_lat_arg" in names[i + 2]]
a = np.array(seq) / 1e3
print(f"{len(a)} steps; lat, gap, gemm2, gap, step (us): median {np.median(a, 0).round(2)} p10 {np.percentile(a, 10, 0).round(2)}")
