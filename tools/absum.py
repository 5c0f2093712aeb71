"""Summary of bench JSON lines in a gpurun_out directory: value, step, rounds, trials, speculative, reruns, k_trial."""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    if "detail" not in d:
        continue
    t = d["detail"]
    print("%-22s %8.1f MB/s %7.1f ms  rounds %4d trials %7d spec %6d rerun %6d ktrial %5.0f kmatch %4.0f kch %4.0f parity %s" % (
        os.path.basename(f)[:-5], d["value"], d["ms_per_step"], t["n_rounds"], t["n_trials"], t["n_trials_speculative"],
        t["n_trials_rerun"], t["k_trial_ms"], t["k_match_ms"], t["k_chains_ms"], (d.get("atz_parity") or {}).get("identical_to_reference")))
