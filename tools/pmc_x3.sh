#!/bin/bash
# PMC passes (kernel-trace only) on fp32 x3 conv kernels: is the hi/lo split VALU the limiter?
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/pmcx3
mkdir -p $R
i=0
IFS=';' read -ra LIST <<< "${SPECS:-128,128,3,1,28 fwd;1024,256,1,1,14 fwd;64,256,1,1,56 fwd;64,64,3,1,56 wgrad;256,256,3,1,14 wgrad;256,1024,1,1,14 wgrad}"
for spec in "${LIST[@]}"; do
  set -- $spec
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" "FETCH_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/p$i -o run -- python3 tools/x3_one.py $1 $2 6 > $R/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/p$i.log; exit 1; }
    echo "$i $1:$2 $grp" >> $R/index.txt
  done
done
find $R -name "*.db" -delete
python3 - <<'PY'
import csv, collections, os
root = "gpurun_out/pmcx3"
index = [l.split(" ", 2) for l in open(os.path.join(root, "index.txt")).read().splitlines()]
res = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for i, shape, grp in index:
    d = os.path.join(root, f"p{i}")
    for f, kind in (("run_counter_collection.csv", "c"), ("run_kernel_trace.csv", "t")):
        path = os.path.join(d, f)
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            if not ("k_conv_x3" in k or "k_conv_wgrad" in k):
                continue
            k = k.split("(")[0][:70]
            if kind == "c":
                res[(shape, k)][r["Counter_Name"]].append(float(r["Counter_Value"]))
            else:
                dur[(shape, k)].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
for (shape, k), cnt in sorted(res.items()):
    m = {c: sum(v) / len(v) for c, v in cnt.items()}
    d = sorted(dur[(shape, k)])[len(dur[(shape, k)]) // 2] / 1e3 if dur[(shape, k)] else 0
    w = m.get("SQ_WAVES", 1)
    line = f"{shape:22s} {k:60s} {d:7.1f} us"
    if "SQ_INSTS_VALU" in m:
        line += f" | per wave VALU {m['SQ_INSTS_VALU'] / w:7.0f} MFMA {m['SQ_INSTS_MFMA'] / w:6.0f} LDS {m['SQ_INSTS_LDS'] / w:6.0f} VMEM {m['SQ_INSTS_VMEM_RD'] / w:5.0f} SALU {m['SQ_INSTS_SALU'] / w:6.0f}"
    if "GRBM_GUI_ACTIVE" in m:
        wall = m["GRBM_GUI_ACTIVE"] / 8
        line += f" | MFMA busy {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (wall * 1024):.3f}"
    if "SQ_WAVE_CYCLES" in m and "SQ_ACTIVE_INST_VALU" in m:
        pass
    if "SQ_WAIT_ANY" in m:
        tot = m["SQ_WAIT_ANY"] + m["SQ_WAIT_INST_ANY"] + m["SQ_ACTIVE_INST_ANY"]
        line += f" | wait {m['SQ_WAIT_ANY'] / tot:.2f} issue-stall {m['SQ_WAIT_INST_ANY'] / tot:.2f} active {m['SQ_ACTIVE_INST_ANY'] / tot:.2f} (VALU {m['SQ_ACTIVE_INST_VALU'] / tot:.2f}) LDS-conf {m['SQ_LDS_BANK_CONFLICT']:.0f}"
    if "FETCH_SIZE" in m:
        line += f" | fetch {2 * m['FETCH_SIZE'] / 1e6:.2f} GB"
    print(line)
PY
