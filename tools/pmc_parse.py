"""Summarise rocprofv3 PMC csvs of tools/pmc_round.sh: per-dispatch mean of every counter for
the step kernel, HBM bytes per launch (gfx950 FETCH_SIZE correction), derived utilisations."""
import csv, glob, json, os, sys
from collections import defaultdict

out = sys.argv[1]
vals = defaultdict(list)
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if "step_kernel" not in row.get("Kernel_Name", ""):
            continue
        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in vals.items() if v}
res = {"counters_mean_per_dispatch": m}
if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
    # FETCH_SIZE/WRITE_SIZE are KiB.  gfx950 FETCH_SIZE counts 128-B reads as 64 B for wide
    # streaming loads (MI355X_MICROARCH.md, HBM); both raw and x2-corrected reads are reported.
    rd_raw = m["FETCH_SIZE"] * 1024
    wr = m["WRITE_SIZE"] * 1024
    res["hbm_read_bytes_raw"] = rd_raw
    res["hbm_read_bytes_x2"] = 2 * rd_raw
    res["hbm_write_bytes"] = wr
if "TCC_EA0_RDREQ_sum" in m:
    res["ea_rd_bytes_64B"] = m["TCC_EA0_RDREQ_sum"] * 64
    res["ea_wr_bytes_64B"] = m.get("TCC_EA0_WRREQ_sum", 0) * 64
if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
    wc = m["SQ_WAVE_CYCLES"]
    res["valu_active_frac_of_wave_cycles"] = m.get("SQ_ACTIVE_INST_VALU", 0) / wc
    res["wait_any_frac"] = m.get("SQ_WAIT_ANY", 0) / wc
    res["wait_inst_any_frac"] = m.get("SQ_WAIT_INST_ANY", 0) / wc
    res["active_inst_any_frac"] = m.get("SQ_ACTIVE_INST_ANY", 0) / wc
if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m:
    res["valu_insts_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
    res["salu_insts_per_wave"] = m.get("SQ_INSTS_SALU", 0) / m["SQ_WAVES"]
    res["vmem_rd_per_wave"] = m.get("SQ_INSTS_VMEM_RD", 0) / m["SQ_WAVES"]
    res["vmem_wr_per_wave"] = m.get("SQ_INSTS_VMEM_WR", 0) / m["SQ_WAVES"]
if "TCC_HIT_sum" in m:
    res["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
json.dump(res, open(os.path.join(out, "pmc_summary.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
