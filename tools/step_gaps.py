"""Busy time, idle gaps and per-kernel totals of the LAST bench step in a rocprofv3 kernel trace.

    python tools/step_gaps.py gpurun_out/tr_lfr1m/tr_kernel_trace.csv [n_steps_total]
The last step starts at the first k_cd_init after the last-but-one run's final-label export
(k_relabel_out); good enough for a warmup+1 trace."""
import collections
import csv
import sys

tr = list(csv.DictReader(open(sys.argv[1])))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(tr) if "k_relabel_out" in r["Kernel_Name"]]
start = ends[-2] + 1 if len(ends) >= 2 else 0
step = tr[start:ends[-1] + 2]
t0 = int(step[0]["Start_Timestamp"]); t1 = max(int(r["End_Timestamp"]) for r in step)
busy = 0; last = t0; big = []; prev = None
tot = collections.Counter(); cnt = collections.Counter()
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s - last > 100000:
        big.append(((s - last) / 1e3, (last - t0) / 1e6, prev["Kernel_Name"][:40], r["Kernel_Name"][:40]))
    busy += max(0, e - max(s, last)); last = max(last, e); prev = r
    tot[r["Kernel_Name"][:70]] += e - s; cnt[r["Kernel_Name"][:70]] += 1
print("step window %.2f ms, GPU busy %.2f ms, %d kernels" % ((t1 - t0) / 1e6, busy / 1e6, len(step)))
for k, v in tot.most_common(30):
    print("%9.3f ms %5d  %s" % (v / 1e6, cnt[k], k))
print("gaps > 100 us:")
for b in big:
    print("  %7.1f us at %7.2f ms after %-42s before %s" % b)
