"""Summarise rocprofv3 --pmc CSV passes (tools/pmc_conv.sh): per shape, per kernel, mean counter
values over dispatches, plus derived MFMA utilisation."""
import collections
import csv
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
index = [l.split(" ", 2) for l in open(os.path.join(root, "index.txt")).read().splitlines()]
res = collections.defaultdict(lambda: collections.defaultdict(list))
for i, shape, grp in index:
    path = os.path.join(root, f"p{i}", "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"][:40]
        if "k_conv" not in k:
            continue
        res[(shape, k)][row["Counter_Name"]].append(float(row["Counter_Value"]))
# kernel durations from the kernel-trace CSVs of the same passes (ns per dispatch)
dur = collections.defaultdict(list)
for i, shape, grp in index:
    path = os.path.join(root, f"p{i}", "run_kernel_trace.csv")
    if not os.path.exists(path):
        continue
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"][:40]
        if "k_conv" in k:
            dur[(shape, k)].append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
for (shape, k), cnt in sorted(res.items()):
    m = {c: sum(v) / len(v) for c, v in cnt.items()}
    print(f"== {shape}  {k}")
    for c in sorted(m):
        print(f"   {c:28s} {m[c]:16.1f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        # SQ_VALU_MFMA_BUSY_CYCLES is summed over all 1024 SIMDs (16 per 16x16x32 MFMA);
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md 'DVFS give-back'), so the
        # kernel's wall cycles are GUI/8 and utilisation = busy / (GUI/8 x 1024) — this reconciles
        # with the measured TF/s ÷ 2.5 PF (the round-1 formula omitted the /8)
        wall = m["GRBM_GUI_ACTIVE"] / 8
        print(f"   MFMA util = {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (wall * 1024):.3f}"
              f"  (busy / (GUI_ACTIVE/8 x 1024 SIMDs)); wall cycles {wall:.0f}")
    if "SQ_INSTS_MFMA" in m and dur.get((shape, k)):
        # reconciliation: every v_mfma_f32_16x16x32_bf16 is 16·16·32·2 FLOP; FLOP / trace duration
        # is the achieved rate, and ÷ 2.5 PF dense bf16 must match the busy-counter utilisation
        d = sorted(dur[(shape, k)])[len(dur[(shape, k)]) // 2]
        fpm = 32768 if "k_conv_x8" in k else 16384  # 32x32x16 vs 16x16x32 bf16 MFMA
        tf = m["SQ_INSTS_MFMA"] * fpm / d / 1e3
        print(f"   median duration {d / 1e3:.1f} us; MFMA FLOP {m['SQ_INSTS_MFMA'] * fpm / 1e9:.2f} GFLOP; "
              f"{tf:.0f} TF/s = {tf / 2500:.3f} of 2.5 PF")
        print(f"   VALU per MFMA = {m['SQ_INSTS_VALU'] / max(m['SQ_INSTS_MFMA'], 1):.2f}")
    if "TCC_HIT_sum" in m:
        print(f"   L2 hit = {m['TCC_HIT_sum'] / max(m['TCC_HIT_sum'] + m['TCC_MISS_sum'], 1):.3f}")
