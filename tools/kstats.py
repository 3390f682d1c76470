"""Print the mapper kernels of a rocprofv3 kernel_stats.csv (skips scan registration + copies)."""
import csv
import sys

for x in csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv")):
    if "k_sr" in x["Name"] or "Buffer" in x["Name"]:
        continue
    print(f"{x['Name'][:48]:48s} {x['Calls']:>6s} {float(x['AverageNs']) / 1e3:9.1f}us "
          f"min {float(x['MinNs']) / 1e3:.1f} max {float(x['MaxNs']) / 1e3:.1f}")
