#!/usr/bin/env python
"""Per-kernel mean counter values per dispatch from tools/gpu_pmc.sh output (rocprofv3 --pmc CSVs), with the
derived shares: wave-cycle split (active / issue-stall / wait), MFMA busy per CU-cycle, instructions per wave.

    python tools/pmc_summary.py gpurun_out/<tag>/pmc [--match conv_]
"""
import argparse
import collections
import csv
import glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{a.root}/pmc*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            if a.match and a.match not in name:
                continue
            key = (name.split("(")[0][:48], int(r["Grid_Size"]) // int(r["Workgroup_Size"]))
            vals[key][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    for key, d in vals.items():
        per = collections.defaultdict(list)
        for (c, _disp), v in d.items():
            per[c].append(sum(v))          # summed over the dimension instances of one dispatch
        m = {c: sum(v) / len(v) for c, v in per.items()}
        wc = m.get("SQ_WAVE_CYCLES", 0) or 1
        waves = m.get("SQ_WAVES", 1) or 1
        out = {"wgs": key[1]}
        if "SQ_WAVE_CYCLES" in m:
            out.update(active=round(m.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3), stall=round(m.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
                       wait=round(m.get("SQ_WAIT_ANY", 0) / wc, 3))
        if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            out["gui_active_cyc"] = round(m["GRBM_GUI_ACTIVE"] / 8)
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
            if c in m:
                out[c.replace("SQ_INSTS_", "") + "/wave"] = round(m[c] / waves, 1)
        for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES",
                  "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC"):
            if c in m:
                out[c.replace("SQ_", "").lower()] = round(m[c])
        print(key[0], out)


if __name__ == "__main__":
    main()
