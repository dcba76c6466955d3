"""Summarise rocprofv3 --pmc counter CSVs per e2ep kernel (mean per dispatch over the passes
of one shape): python scripts/pmc_table.py <dir with *_p1, *_p2, *_fetch, *_write> <shape>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    rows = defaultdict(lambda: defaultdict(list))
    vg = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"]
                if "e2ep::" not in k:
                    continue
                k = k.split("(")[0].replace("void ", "")
                rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                vg[k] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"])
    return rows, vg


def main():
    base, shape = sys.argv[1], sys.argv[2]
    out = defaultdict(dict)
    vgs = {}
    for p in ("p1", "p2", "fetch", "write"):
        rows, vg = load(os.path.join(base, f"{shape}_{p}"))
        vgs.update(vg)
        for k, cs in rows.items():
            for c, v in cs.items():
                out[k][c] = sum(v) / len(v)
    for k, cs in out.items():
        print(f"== {shape}: {k}  (VGPR, AGPR, SGPR, LDS) = {vgs.get(k)}")
        for c in sorted(cs):
            print(f"   {c:28s} {cs[c]:16.1f}")
        if "SQ_WAVE_CYCLES" in cs and cs["SQ_WAVE_CYCLES"] > 0:
            wc = cs["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in cs:
                    print(f"   {c + ' / WAVE_CYCLES':40s} {cs[c] / wc:8.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and cs.get("GRBM_GUI_ACTIVE"):
            # MFMA busy is summed over all 1024 SIMDs (64 cycles per fp32 32x32x2 MFMA, i.e.
            # 64 FLOP / SIMD / cycle = the 157.3 TF peak at 2.4 GHz); GRBM_GUI_ACTIVE is
            # summed over the 8 XCDs, so one XCD's active cycles = GRBM / 8.
            util = cs["SQ_VALU_MFMA_BUSY_CYCLES"] / (cs["GRBM_GUI_ACTIVE"] / 8 * 1024)
            print(f"   {'MFMA utilisation (busy / (GRBM/8 x 1024))':40s} {util:8.3f}")
            print(f"   {'MFMA FLOP issued (busy x 64), GFLOP':40s} "
                  f"{cs['SQ_VALU_MFMA_BUSY_CYCLES'] * 64 / 1e9:8.2f}")
            print(f"   {'kernel time (GRBM/8 / 2.4 GHz), us':40s} "
                  f"{cs['GRBM_GUI_ACTIVE'] / 8 / 2.4e3:8.1f}")
        if "FETCH_SIZE" in cs:
            print(f"   {'HBM read (FETCH_SIZE x2, KB->MB)':40s} {2 * cs['FETCH_SIZE'] / 1e3:8.1f}")
        if "WRITE_SIZE" in cs:
            print(f"   {'HBM write (WRITE_SIZE, KB->MB)':40s} {cs['WRITE_SIZE'] / 1e3:8.1f}")


if __name__ == "__main__":
    main()
