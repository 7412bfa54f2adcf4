#!/usr/bin/env python3
"""Per-kernel SQ counter ratios from the two rocprofv3 passes of
tools/gpu_sqpmc.sh.

    python tools/sq_summary.py gpurun_out/<tag> [kernel-substring]

MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * CUs) (per-CU
busy fraction); wait_any / wait_inst_any / active_inst are per wave-cycle
(divided by SQ_WAVE_CYCLES); instruction counts are per wave launched."""
import collections
import csv
import glob
import os
import sys

CUS = 256


def load(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    data = collections.defaultdict(dict)
    for sub in ("a", "b"):
        for k, cs in load(os.path.join(root, sub)).items():
            for c, v in cs.items():
                data[k][c] = sum(v) / len(v)
    for k, c in sorted(data.items()):
        if filt not in k:
            continue
        g = lambda n: c.get(n, float("nan"))
        wc = g("SQ_WAVE_CYCLES")
        print(k[:90])
        print(f"  mfma_busy {g('SQ_VALU_MFMA_BUSY_CYCLES') / (g('GRBM_GUI_ACTIVE') * CUS):.3f}"
              f"  wait_any {g('SQ_WAIT_ANY') / wc:.3f}  wait_inst_any {g('SQ_WAIT_INST_ANY') / wc:.3f}"
              f"  active_inst {g('SQ_ACTIVE_INST_ANY') / wc:.3f}  wait_lds {g('SQ_WAIT_INST_LDS') / wc:.3f}"
              f"  lds_conflict {g('SQ_LDS_BANK_CONFLICT'):.3g}")
        print(f"  insts: mfma {g('SQ_INSTS_MFMA'):.4g} valu {g('SQ_INSTS_VALU'):.4g} lds {g('SQ_INSTS_LDS'):.4g}"
              f" salu {g('SQ_INSTS_SALU'):.4g}  vmem_rd_cycles {g('SQ_INST_CYCLES_VMEM_RD'):.4g}"
              f"  gui_active {g('GRBM_GUI_ACTIVE'):.4g}")


if __name__ == "__main__":
    main()
