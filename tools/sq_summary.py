"""Per-kernel SQ counter summary of rocprofv3 --pmc runs (tools/pmc_sq.sh):
fractions of wave cycles active / waiting (s_waitcnt, barrier) / issue-stalled,
VALU-active fraction, instructions per wave.  usage: sq_summary.py DIR..."""
import collections
import csv
import re
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        if not m or not m.group(1).startswith("k_cg"):
            continue
        k = m.group(1)
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        acc[k]["vgpr"] = [int(r["VGPR_Count"])]
    for k, c in sorted(acc.items()):
        a = {n: sum(x) / len(x) for n, x in c.items()}
        wc, nw = a["SQ_WAVE_CYCLES"], max(a["SQ_WAVES"], 1)
        print("%s %-28s n=%3d vgpr=%3d waves=%6.0f active %.2f wait %.2f stall %.2f valu %.2f "
              "| per wave: VALU %5.0f LDS %4.0f quadcyc %6.0f"
              % (d.split("/")[-1], k, len(c["SQ_WAVES"]), a["vgpr"], nw, a["SQ_ACTIVE_INST_ANY"] / wc,
                 a["SQ_WAIT_ANY"] / wc, a["SQ_WAIT_INST_ANY"] / wc, a["SQ_ACTIVE_INST_VALU"] / wc,
                 a["SQ_INSTS_VALU"] / nw, a["SQ_INSTS_LDS"] / nw, wc / nw))
