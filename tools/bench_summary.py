"""Print the key numbers of bench JSON lines found in gpurun_out/*.log."""
import json
import sys

for f in sys.argv[1:]:
    try:
        line = [l for l in open(f) if l.startswith("{")][-1]
    except (OSError, IndexError) as e:
        print(f, "no JSON line", e)
        continue
    d = json.loads(line)
    r = d["roofline"]
    print("%s: %.5g %s  roofline %s %.1f GB/s (%.3f)  iter %.5f ms %.1f GB/s" % (
        f, d["value"], d["unit"], r["kernel"].split()[0], r["achieved"], r["frac"],
        d["cg_iteration"]["ms"], d["cg_iteration"]["gbs"]))
    for k, v in d["cg_kernels"].items():
        print("   %-6s %.5f ms %7.1f GB/s  x%d" % (k, v["avg_launch_ms"], v["gbs"], v["launches"]))
    for fm, row in d.get("kernel_probe", {}).items():
        print("   probe %-8s" % fm, "  ".join("%s %.4f/%.0f" % (k, v["ms"], v["gbs"])
                                            for k, v in row.items()))
    if "cpu_baseline" in d:
        print("   cpu", d["cpu_baseline"])
