"""Sum rocprofv3 counter_collection rows of the kernels whose name contains SUBSTR, per
counter, over every pass directory under ROOT (tools/gpu_pmc_kernel.sh).

    python tools/pmc_kernel.py gpurun_out/pmck_TAG swin_attn_kernel<96
"""
import csv
import glob
import sys
from collections import defaultdict


def main(root, sub):
    tot = defaultdict(float)
    disp = defaultdict(set)
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add(r.get("Dispatch_Id", ""))
    for k in sorted(tot):
        print(f"{k:28s} {tot[k]:16.4g}  ({len(disp[k])} dispatches)")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
