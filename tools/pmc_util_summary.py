"""Summarise tools/gpu_pmc_util.sh runs: per (case, kernel) MFMA busy %, LDS busy %, bank conflicts.

MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * 1024 SIMDs); LDS util = SQ_LDS_IDX_ACTIVE /
(GRBM_GUI_ACTIVE * 256 CUs) (rocprofv3's MfmaUtil / LdsUtil derived-counter expressions).
"""
import collections
import csv
import glob
import os
import sys


def main():
    for d in sys.argv[1:]:
        if not os.path.isdir(d):
            continue
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            rows += list(csv.DictReader(open(f)))
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        cnt = collections.Counter()
        for r in rows:
            k = (r["Kernel_Name"][:70], r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        per_kernel = collections.defaultdict(list)
        for (name, _), ctr in agg.items():
            per_kernel[name].append(ctr)
        print(os.path.basename(d))
        for name, lst in per_kernel.items():
            def avg(c):
                return sum(x.get(c, 0.0) for x in lst) / len(lst)
            gui = avg("GRBM_GUI_ACTIVE") or 1.0
            mf = 100 * avg("SQ_VALU_MFMA_BUSY_CYCLES") / (gui * 1024)
            lds = 100 * avg("SQ_LDS_IDX_ACTIVE") / (gui * 256)
            bc = avg("SQ_LDS_BANK_CONFLICT") / max(1.0, avg("SQ_LDS_IDX_ACTIVE"))
            print(f"   {name:70s} n={len(lst)} MFMA {mf:5.1f}%  LDS {lds:5.1f}%  bank-conflict {100 * bc:4.1f}%  "
                  f"LDS insts {avg('SQ_INSTS_LDS'):.3g}  MFMA insts {avg('SQ_INSTS_MFMA'):.3g}")


if __name__ == "__main__":
    main()
