"""Short summary of a rocprofv3 kernel_stats.csv: the engine's kernels (zrx::), calls and
average / min / max microseconds.  usage: python scripts/kstats.py <kernel_stats.csv> ..."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print(path)
    for r in csv.DictReader(open(path)):
        n = r["Name"]
        if "zrx::" not in n:
            continue
        short = re.sub(r"\(.*", "", n.replace("void ", "").replace("zrx::", ""))
        print(f"  {short:34s} calls {int(r['Calls']):5d}  avg {float(r['AverageNs']) / 1e3:9.2f} us  "
              f"min {float(r['MinNs']) / 1e3:9.2f}  max {float(r['MaxNs']) / 1e3:9.2f}")
