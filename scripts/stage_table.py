"""Stage budget of the scan forms of one config from scripts/r05_stage.sh outputs (forms.json of
one or more stage directories): per ablation variant and kernel form, the traced median and the
PMC counters, ordered as the stages build up, with each stage's increment over the one before.
usage: python scripts/stage_table.py <out.json> <config> <stage dir> [<stage dir> ...]"""
import json
import os
import sys

# variant -> what the scan does in it (scripts/ablate_variants.py); ordered as the stages add up
STAGES = [
    (5, "stream the packed genome, validity masks, super-step claims (no filter)"),
    (1, "+ level-1 LDS filter (word + 2-bit test per window)"),
    (2, "+ candidate list (ballot compaction of level-1 survivors)"),
    (3, "+ level-2 L2 loads (exact bucket bitmap / key-group words)"),
    (6, "+ key-group field test and compaction, no key-reference writes"),
    (0, "product (key-reference writes included)"),
]
KEYS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "TCC_HIT_sum",
        "TCC_MISS_sum")

out, cfg, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
rows = {}
for d in dirs:
    forms = json.load(open(os.path.join(d, "forms.json")))
    for path, kernels in forms.items():
        base = os.path.basename(path)
        if base.endswith(".log"):
            continue
        v = int(base[1:])
        for name, vals in kernels.items():
            if "scan_kernel" not in name and "dense_kernel" not in name:
                continue
            r = rows.setdefault(name, {}).setdefault(v, {})
            if base[0] == "t":
                r["median_us"], r["min_us"] = vals["median_us"], vals["min_us"]
            else:
                r.update({k: vals[k] for k in KEYS if k in vals})
table = {"config": cfg, "sources": dirs,
         "note": "timing-only ablations (scripts/ablate_variants.py), each variant in its own process under a "
                 "kernel trace, then one PMC pass (scripts/r05_stage.sh); counters are per launch, summed over "
                 "the chip; 'delta_us' is the increment over the stage before",
         "forms": {}}
for name, per in rows.items():
    prev = None
    stages = []
    for v, what in STAGES:
        if v not in per:
            continue
        r = dict(variant=v, stage=what, **per[v])
        if prev is not None and "median_us" in r and "median_us" in prev:
            r["delta_us"] = round(r["median_us"] - prev["median_us"], 1)
        stages.append(r)
        prev = r
    table["forms"][name] = stages
json.dump(table, open(out, "w"), indent=1)
for name, stages in table["forms"].items():
    print(name)
    for r in stages:
        print(f"  v{r['variant']:<2d} {r.get('median_us', float('nan')):8.1f} us  d {r.get('delta_us', 0):7.1f}  "
              f"VALU {r.get('SQ_INSTS_VALU', 0):.3e}  {r['stage']}")
