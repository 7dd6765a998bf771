#!/usr/bin/env python3
"""GPU idle time between kernels in a rocprofv3 kernel trace (--kernel-trace, csv): how much of
a latency-bound run (e.g. one GPU's n_p = 8 share) is kernel-boundary gaps rather than kernel
time.  Gaps longer than --host-ms are reported apart (host phases: graph generation, timing
boundaries).  Usage: tools/trace_gaps.py <kernel_trace.csv> [--host-ms 2]"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--host-ms", type=float, default=2.0)
    args = ap.parse_args()
    ks = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    busy, gaps, host, per = 0, defaultdict(int), 0, defaultdict(lambda: [0, 0])
    end = ks[0][0]
    for s, e, name in ks:
        short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        short = short.split("<")[0] + ("<" + short.split("<", 1)[1] if "<" in short else "")
        per[short[:70]][0] += e - s
        per[short[:70]][1] += 1
        if s > end:
            g = s - end
            if g > args.host_ms * 1e6:
                host += g
            else:
                b = "<2us" if g < 2000 else "2-5us" if g < 5000 else "5-10us" if g < 10000 else \
                    "10-50us" if g < 50000 else ">50us"
                gaps[b] += g
        busy += max(0, e - max(s, end))
        end = max(end, e)
    span = end - ks[0][0] - host
    print("kernels %d, span without host phases %.1f ms, kernel-busy %.1f ms (%.0f%%), gaps %.1f ms"
          % (len(ks), span / 1e6, busy / 1e6, 100.0 * busy / span, sum(gaps.values()) / 1e6))
    for b in ("<2us", "2-5us", "5-10us", "10-50us", ">50us"):
        print("  gaps %-8s %.2f ms" % (b, gaps[b] / 1e6))
    print("host phases (gaps > %.1f ms): %.1f ms" % (args.host_ms, host / 1e6))
    for name, (t, c) in sorted(per.items(), key=lambda x: -x[1][0])[:30]:
        print("  %8.2f ms %6d  %s" % (t / 1e6, c, name))


if __name__ == "__main__":
    main()
