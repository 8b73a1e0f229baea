#!/bin/bash
# Dynamic VALU instruction mix per kernel (two --pmc passes, kernel trace only).
set -o pipefail
TAG=${1:-mix}
shift
OUT=gpurun_out/$TAG/mix
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64" "SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-f32-leg "$@" > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i ($grp) failed"; tail -5 $OUT/p$i.err; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(dict))
for f in sorted(glob.glob(f"{out}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void gk::", "")
        if "gk::" not in r["Kernel_Name"]:
            continue
        d = vals[k][r["Counter_Name"]]
        d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
for k, cs in vals.items():
    m = {c: sum(v.values()) / len(v) for c, v in cs.items()}
    if m.get("SQ_INSTS_VALU", 0) < 1e6:
        continue
    v = m["SQ_INSTS_VALU"]
    f64 = sum(m.get(c, 0) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
    print(f"{k[:60]:60s} VALU {v:.3g}  f64 {f64/v:.1%} (add {m.get('SQ_INSTS_VALU_ADD_F64',0)/v:.1%} mul {m.get('SQ_INSTS_VALU_MUL_F64',0)/v:.1%} fma {m.get('SQ_INSTS_VALU_FMA_F64',0)/v:.1%} trans {m.get('SQ_INSTS_VALU_TRANS_F64',0)/v:.1%})"
          f"  int32 {m.get('SQ_INSTS_VALU_INT32',0)/v:.1%} int64 {m.get('SQ_INSTS_VALU_INT64',0)/v:.1%} cvt {m.get('SQ_INSTS_VALU_CVT',0)/v:.1%}"
          f"  SALU {m.get('SQ_INSTS_SALU',0):.3g} LDS {m.get('SQ_INSTS_LDS',0):.3g} VALUactive/wavecyc {m.get('SQ_ACTIVE_INST_VALU',0)/max(m.get('SQ_WAVE_CYCLES',1),1):.2f}")
PY
