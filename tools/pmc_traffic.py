"""HBM traffic per launch from rocprofv3 PMC passes (tools/gpu_pmc.sh with
FETCH_SIZE and WRITE_SIZE passes) -> profiles/pmc_<tag>.json.

Correction (MI355X_MICROARCH.md, HBM): on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced streaming read -> doubled; WRITE_SIZE is exact for
16-B-per-lane stores (8-B stores are uncalibrated: reported as measured).
Both counters are in KiB."""
import collections
import csv
import glob
import json
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
out = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/pmc_summary.json"
KEYS = {"ppo_step": r"ppo_step_kernel", "ppo_rows16": r"ppo_rows16_kernel(<false|ILb0)", "ppo_rows16_metrics": r"ppo_rows16_kernel(<true|ILb1)", "wgrad": r"wgrad_kernel", "policy_step": r"policy_step_kernel", "policy_rollout": r"policy_rollout_kernel",
        "gae": r"gae_kernel", "reduce_grads": r"reduce_grads_kernel", "env_step": r"env_step_kernel",
        "adam": r"adam_kernel", "project": r"project_kernel", "sumsq": r"sumsq_partial_kernel",
        "optim": r"optim_fused_kernel", "lstm_fwd_step": r"lstm_fwd_step", "lstm_bwd_step": r"lstm_bwd_step",
        "lstm_gin": r"lstm_gin_kernel", "rollout16": r"rollout16_kernel", "lstm_dfeat": r"lstm_dfeat_kernel"}
vals = collections.defaultdict(lambda: collections.defaultdict(list))
names = {}
for f in sorted(glob.glob(f"{root}/p*/*counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        for key, pat in KEYS.items():
            if re.search(pat, row["Kernel_Name"]):
                vals[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
                names[key] = row["Kernel_Name"]
res = {}
for key, cs in vals.items():
    d = {c: sum(v) / len(v) for c, v in cs.items()}
    fetch = d.get("FETCH_SIZE")
    write = d.get("WRITE_SIZE")
    ent = {"kernel_name": names[key], "counters_avg_per_launch": d, "launches": {c: len(v) for c, v in cs.items()}}
    busy, gui = d.get("SQ_VALU_MFMA_BUSY_CYCLES"), d.get("GRBM_GUI_ACTIVE")
    if busy is not None and gui:
        # MfmaUtil (rocprofv3's derived formula): MFMA-busy cycles over the
        # kernel's active cycles x 1 024 SIMDs; GRBM_GUI_ACTIVE comes summed
        # over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back) -> / 8
        ent["mfma_busy_frac"] = busy / (gui / 8 * 1024)
        ent["active_cycles_per_xcd"] = gui / 8
    if fetch is not None and write is not None:
        ent["hbm_read_bytes_per_launch"] = 2 * fetch * 1024
        ent["hbm_write_bytes_per_launch"] = write * 1024
        ent["hbm_bytes_per_launch"] = 2 * fetch * 1024 + write * 1024
    res[key] = ent
json.dump({"source": root, "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE as is; KiB->B; "
           "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)",
           "kernels": res}, open(out, "w"), indent=1)
print(json.dumps({k: v.get("hbm_bytes_per_launch") for k, v in res.items()}))
