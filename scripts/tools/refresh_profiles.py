"""Copy one scripts/profile_round.sh run (gpurun_out/<R>_*) into profiles/<ROUND>/ and recompute
profiles/traffic_fingerprint.json from its PMC passes.

Usage: python scripts/tools/refresh_profiles.py R WARMUP STEPS KERNEL_BUILD_NOTE
  R        the profile_round.sh tag (gpurun_out/R_trace, R_pmc_FETCH_SIZE, R_pmc_WRITE_SIZE)
  WARMUP, STEPS  the bench arguments of the traced run (C2 dispatch selection)
  ROUND (env, default r02): the profiles/ subdirectory the summaries go to
HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB), per MI355X_MICROARCH.md's gfx950
correction for 16-B/lane streaming reads; averaged over the C2-sized dispatches."""
import csv
import re
import json
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
R, warm, steps, note = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
src = os.path.join(REPO, "gpurun_out")
ROUND = os.environ.get("ROUND", "r02")
dst = os.path.join(REPO, "profiles", ROUND)
os.makedirs(dst, exist_ok=True)
C2_FRAMES = 960512

for f in ("bench_kernel_stats.csv", "bench_kernel_trace.csv", "bench_domain_stats.csv"):
    shutil.copy(os.path.join(src, R + "_trace", f), os.path.join(dst, f))
shutil.copy(os.path.join(src, R + "_trace.json"), os.path.join(dst, "bench_under_rocprof.json"))
# untimed steps before the timed ones: --warmup plus bench.py's clock warm-up steps
warm = str(int(warm) + json.load(open(os.path.join(dst, "bench_under_rocprof.json"))).get("clock_warmup_steps", 0))
subprocess.run([sys.executable, os.path.join(REPO, "scripts", "tools", "c2_dispatches.py"),
                os.path.join(dst, "bench_kernel_trace.csv"), warm, steps,
                os.path.join(dst, "fingerprint_c2_dispatches.csv")], check=True)


FIN_GRID = min(8192, (2 * C2_FRAMES + 255) // 256) * 256  # finish_db_kernel's grid for a C2 step


def pmc(counter):
    """Mean counter value per C2 step: fingerprint kernel (largest grid) + its finish_db_kernel."""
    path = os.path.join(src, "%s_pmc_%s" % (R, counter), "run_counter_collection.csv")
    shutil.copy(path, os.path.join(dst, "pmc_%s.csv" % counter))
    rows = list(csv.DictReader(open(path)))
    fp = [r for r in rows if re.search(r"fingerprint(8k)?_kernel", r["Kernel_Name"])]
    grid = max(int(r["Grid_Size"]) for r in fp)
    vals = [float(r["Counter_Value"]) for r in fp if int(r["Grid_Size"]) == grid]
    fin = [float(r["Counter_Value"]) for r in rows
           if "finish_db_kernel" in r["Kernel_Name"] and int(r["Grid_Size"]) == FIN_GRID]
    return sum(vals) / len(vals) + (sum(fin) / len(fin) if fin else 0.0)


fetch_kb, write_kb = pmc("FETCH_SIZE"), pmc("WRITE_SIZE")
hbm = (2 * fetch_kb + write_kb) * 1024.0
alg = 520 * C2_FRAMES
out = {
    "kernel": "fingerprint8k_kernel + finish_db_kernel (one C2 step)",
    "frames_per_launch": C2_FRAMES,
    "hbm_bytes_per_launch": hbm,
    "fetch_size_kb_raw": fetch_kb,
    "write_size_kb_raw": write_kb,
    "algorithmic_bytes_per_launch": alg,
    "traffic_over_algorithmic": hbm / alg,
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (scripts/profile_round.sh); "
              "FETCH_SIZE x2: MI355X_MICROARCH.md's HBM section gives the factor for 16-B/lane streaming reads, "
              "and the kernel's 4-B buffer-load pattern was calibrated on the box in round 5 against a 512 MiB "
              "buffer read once (scripts/microbench/fetch_calib.hip: 262.3 MB reported for the dword pattern, "
              "256.0 MB for a 16-B stream: the same factor 2); WRITE_SIZE as reported (uncalibrated for 4-B "
              "scattered stores)",
    "round": ROUND,
    "kernel_build": note,
}
json.dump(out, open(os.path.join(REPO, "profiles", "traffic_fingerprint.json"), "w"), indent=1)
print("traffic %.1f MB/launch = %.3f x algorithmic" % (hbm / 1e6, hbm / alg))
