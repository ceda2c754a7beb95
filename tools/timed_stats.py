#!/usr/bin/env python3
"""The rocprofv3 statistics of bench.py's TIMED launches only (VERDICT r04 weak 4:
the --stats summary of a bench run averages the placement-search probes, the
first step, the prewarm and the energy window together with the timed steps).

The bench line says how many KSEG launches come before the timed ones:
placement.launches (the search's probes, warm-ups included) + 1 (first_step_ms)
+ prewarm_steps; then `steps` timed launches.  In dispatch order those are the
launches [before, before + steps) of the physics kernel in the kernel trace.
Writes a stats CSV in rocprofv3's column layout for those launches and their
durations, and prints the mean against the bench line's kernel_ms.

usage: timed_stats.py <kernel_trace.csv> <bench_json_line_file> <out_prefix> [kernel_regex]"""
import csv
import json
import re
import statistics as stt
import sys


def main():
    trace, bench, out = sys.argv[1:4]
    regex = sys.argv[4] if len(sys.argv) > 4 else "kseg_entry"
    line = [json.loads(x) for x in open(bench) if x.startswith("{")][-1]
    before = line["placement"]["launches"] + 1 + line["prewarm_steps"]
    steps = line["steps"]
    rows = [r for r in csv.DictReader(open(trace)) if re.search(regex, r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    timed = rows[before:before + steps]
    if len(timed) != steps:
        sys.exit("only %d of %d timed launches in the trace (%d launches, %d before)" % (len(timed), steps, len(rows),
                                                                                          before))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in timed]
    name = timed[0]["Kernel_Name"]
    with open(out + "_timed_stats.csv", "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        w.writerow([name, len(d), sum(d), sum(d) / len(d), 100.0, min(d), max(d), stt.pstdev(d)])
    with open(out + "_timed_durations.txt", "w") as fh:
        fh.write("# %s: the %d timed launches of the bench (dispatches %d..%d of %d in start order), ns\n"
                 % (name, len(d), before, before + steps - 1, len(rows)))
        fh.write("\n".join(str(x) for x in d) + "\n")
    print(json.dumps({"kernel": name[:60], "launches_in_trace": len(rows), "timed_from": before, "timed": len(d),
                      "rocprof_mean_ms": round(sum(d) / len(d) * 1e-6, 4),
                      "rocprof_median_ms": round(stt.median(d) * 1e-6, 4),
                      "bench_kernel_ms": line["kernel_ms"], "bench_kernel_ms_median": line["kernel_ms_median"]}))


if __name__ == "__main__":
    main()
