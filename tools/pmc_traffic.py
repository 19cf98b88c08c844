"""Turn the PMC passes of tools/pmc_traffic.sh into per-launch HBM bytes of the step kernel.

Calibration: membench's SoA kernel (R84 W72 + obs34, N=262144) moves a known number of bytes
with the step kernel's access width (4 B per lane, 256 B per wave instruction; obs rows as
8-B stores at a 136-B stride).  bytes/counter ratios from it convert the step kernel's FETCH_SIZE /
WRITE_SIZE (KiB) into bytes.  Writes profiles/step_kernel_traffic.json for bench.py."""
import csv, glob, json, os, sys

out = sys.argv[1]
N_STEP = int(sys.argv[2]) if len(sys.argv) > 2 else 262144      # envs of the profiled bench run
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


TAIL = 30   # the timed launches: the last 30 dispatches (bench.py --steps 30 after the warm-up)


def mean_counter(d, name, kern, tail=TAIL):
    """Mean per dispatch over the last `tail` dispatches of `kern` (0 = all) at the largest grid
    of the pass (the workload's launches: bench.py's other keys may launch the kernel on fewer
    envs); a dispatch's counter may come as several rows (per XCD / dimension), which are summed."""
    per, grid = {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for i, row in enumerate(csv.DictReader(open(f))):
            if kern in row.get("Kernel_Name", "") and row["Counter_Name"] == name:
                key = int(row.get("Dispatch_Id") or i)
                per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
                grid[key] = int(row.get("Grid_Size") or 0)
    if not per:
        raise SystemExit(f"no {name} samples for {kern} in {d}")
    g = max(grid.values())
    v = [per[k] for k in sorted(per) if grid[k] == g][-tail if tail else 0:]
    return sum(v) / len(v)


def kernel_key():
    sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))
    from cf2sim.build import _obj_key
    return _obj_key("cf2sim_kernels.hip")


N = 262144
calib_rd = N * 4 * 84
calib_wr = N * 4 * (72 + 34)
c_f = mean_counter(os.path.join(out, "calib_FETCH_SIZE"), "FETCH_SIZE", "kern", 0) * 1024
c_w = mean_counter(os.path.join(out, "calib_WRITE_SIZE"), "WRITE_SIZE", "kern", 0) * 1024
s_f = mean_counter(os.path.join(out, "step_FETCH_SIZE"), "FETCH_SIZE", "step_kernel") * 1024
s_w = mean_counter(os.path.join(out, "step_WRITE_SIZE"), "WRITE_SIZE", "step_kernel") * 1024
kr, kw = calib_rd / c_f, calib_wr / c_w
res = {
    "workload": f"DroneHoverBulletFreeEnvWithGust-v0:N={N_STEP}",
    "hbm_bytes_per_launch": s_f * kr + s_w * kw,
    "read_bytes_per_launch": s_f * kr,
    "write_bytes_per_launch": s_w * kw,
    "raw_FETCH_SIZE_bytes": s_f, "raw_WRITE_SIZE_bytes": s_w,
    "calibration": {"kernel": "tools/membench.hip SoA R84 W72 +obs34 (4 B/lane)", "known_read_bytes": calib_rd,
                    "known_write_bytes": calib_wr, "FETCH_SIZE_bytes": c_f, "WRITE_SIZE_bytes": c_w,
                    "read_factor": kr, "write_factor": kw},
    "kernel_key": kernel_key(),
    "note": "FETCH_SIZE/WRITE_SIZE count L2 memory-side requests; Infinity-Cache hits are counted "
            "(MI355X_MICROARCH.md HBM section), so this is L2->fabric traffic.",
}
# merged into profiles/step_kernel_traffic.json by workload (one entry per measured env count)
prof = os.path.join(ROOT, "profiles", "step_kernel_traffic.json")
try:
    old = json.load(open(prof))
    entries = old.get("entries", [old])
except (OSError, ValueError):
    entries = []
entries = [e for e in entries if e.get("workload") != res["workload"]] + [res]
json.dump({"entries": entries}, open(os.path.join(out, "step_kernel_traffic.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
