# Round 6, final sources: the read-factor calibrations at the kernels' own launch shapes
# (tools/calib/run_calib_r6.sh), then the PMC records of every config's dominant kernel
# in the init regime (the chain the reference runs) and of configs 2-4 from uniform
# starts (tools/gpu/r6_pmc.sh), with those calibrations in place.
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 bash tools/calib/run_calib_r6.sh > gpurun_out/calib_r6.log 2>&1 || { tail -5 gpurun_out/calib_r6.log; exit 1; }
mkdir -p profiles/r6 && cp gpurun_out/calib_r6/calib_sweep.json gpurun_out/calib_r6/calib_live.json profiles/r6/
bash tools/gpu/r6_pmc.sh cfg2:init:gs_sweep_kernel cfg5:init:gs_sweep_kernel cfg3:init:gs_sweep_long_kernel \
  cfg4:init:gs_sweep_live_kernel cfg2:uniform:gs_sweep_bg_kernel cfg3:uniform:gs_sweep_bg_kernel \
  cfg4:uniform:gs_sweep_bg_kernel ${EXTRA_PMC:-} || exit $?
# (in place for the bench runs that follow in the same call)
cp gpurun_out/r6pmc/pmc_*.json gpurun_out/r6pmc/*_summary.txt profiles/r6/
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6pmc/pmc_*.json")):
    r = json.load(open(f))
    c = r["counters_per_launch"]
    print(f.split("/")[-1], r.get("instantiation", "")[:40], round(r["avg_duration_ns_under_pmc"] / 1e3, 1), "us",
          "traffic", round(r.get("traffic_bytes_per_launch", 0) / 1e6, 2), "MB",
          "W", round(c.get("WRITE_SIZE", 0) * 1024 / 1e6, 2), "MB", "valu", round(r.get("valu", {}).get("frac", 0), 3))
PY
