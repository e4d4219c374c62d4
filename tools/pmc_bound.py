#!/usr/bin/env python3
"""What binds a kernel, from cycle counters (tools/pmc.sh bound): per full-size dispatch of the named
kernel, each pass's counters summed over their rows (XCDs / instances), then the median over the
dispatches of one pass; a counter collected in several passes is read from the first.

Derived figures (MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_WAIT_* count quad-cycles; GRBM_GUI_ACTIVE
is summed over the 8 XCDs, so kernel cycles = GRBM_GUI_ACTIVE / 8). On this stack SQ_ACTIVE_INST_VALU
and SQ_ACTIVE_INST_SCA return instruction counts (equal to SQ_INSTS_VALU / within 2 % of
SQ_INSTS_SALU), not busy cycles, so no busy-cycle fraction is derived from them; the issue-count
forms are:
  valu_issue     SQ_INSTS_VALU * 2 / (SIMDs * kernel cycles)   a wave64 instruction at full rate = 2
                 cycles of a SIMD-32 (three-operand forms take ~2x: profiles/r4_valu_rate.log)
  salu_issue     SQ_INSTS_SALU / (CUs * kernel cycles)          one scalar instruction per CU per cycle
  lds_issue      SQ_INSTS_LDS / (CUs * kernel cycles)           one LDS instruction per CU per cycle
  wait_frac      SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES              wave time waiting on a dependency
  active_frac    SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES            wave time issuing
  waves_per_simd SQ_WAVE_CYCLES * 4 / (SIMDs * kernel cycles)   achieved resident waves
  lds_conflict   SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS      conflict cycles per LDS-active cycle
  ta_busy        TA_TA_BUSY_sum / (CUs * kernel cycles)         the texture addresser (one per CU)
  ta_stalled_by_tc  TA_ADDR_STALLED_BY_TC_CYCLES_sum / (CUs * kernel cycles)
  tcp_pending_stall TCP_PENDING_STALL_CYCLES_sum / (CUs * kernel cycles)   the vector L1 waiting on
                 data pending from the L2

usage: tools/pmc_bound.py PMC_DIR KERNEL_SUBSTRING MIN_GRID [MEASURED_NOTE] > out.json
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

d, kname, min_grid = sys.argv[1], sys.argv[2], int(sys.argv[3])
CUS, SIMDS = 256, 1024
vals = {}  # counter -> median over this pass's dispatches (first pass holding it)
durs = []
for pdir in sorted(glob.glob(os.path.join(d, "p*")), key=lambda x: int(os.path.basename(x)[1:]) if os.path.basename(x)[1:].isdigit() else 0):
    if not os.path.isdir(pdir):
        continue
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(pdir + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if kname not in row["Kernel_Name"]:
                continue
            grid = int(row["Grid_Size"]) if "Grid_Size" in row else int(row["Grid_Size_X"])
            if grid < min_grid:
                continue
            per[row["Counter_Name"]][(f, int(row["Dispatch_Id"]))] += float(row["Counter_Value"])
    for c, by in per.items():
        if c not in vals:
            vals[c] = statistics.median(by.values())
    for f in glob.glob(pdir + "/**/*kernel_trace.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if kname in row["Kernel_Name"]:
                g = int(row.get("Grid_Size") or row.get("Grid_Size_X") or 0)
                if g >= min_grid:
                    durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
out = {"kernel": kname, "counters": vals}
if len(sys.argv) > 4:
    out["measured"] = sys.argv[4]
if durs:
    out["dispatch_ms_median"] = statistics.median(durs)
g = vals.get("GRBM_GUI_ACTIVE")
if g:
    kc = g / 8.0
    out["kernel_cycles"] = kc
    if durs:
        out["effective_clock_GHz"] = kc / (statistics.median(durs) * 1e-3) / 1e9
    der = {}
    if "SQ_INSTS_VALU" in vals:
        der["valu_issue"] = vals["SQ_INSTS_VALU"] * 2 / (SIMDS * kc)
    if "SQ_INSTS_SALU" in vals:
        der["salu_issue"] = vals["SQ_INSTS_SALU"] / (CUS * kc)
    if "SQ_INSTS_LDS" in vals:
        der["lds_issue"] = vals["SQ_INSTS_LDS"] / (CUS * kc)
    if "SQ_WAVE_CYCLES" in vals:
        der["waves_per_simd"] = vals["SQ_WAVE_CYCLES"] * 4 / (SIMDS * kc)
        if "SQ_WAIT_INST_ANY" in vals:
            der["wait_frac"] = vals["SQ_WAIT_INST_ANY"] / vals["SQ_WAVE_CYCLES"]
        if "SQ_ACTIVE_INST_ANY" in vals:
            der["active_frac"] = vals["SQ_ACTIVE_INST_ANY"] / vals["SQ_WAVE_CYCLES"]
    if "SQ_LDS_BANK_CONFLICT" in vals and vals.get("SQ_ACTIVE_INST_LDS"):
        der["lds_conflict"] = vals["SQ_LDS_BANK_CONFLICT"] / vals["SQ_ACTIVE_INST_LDS"]
    if "TA_TA_BUSY_sum" in vals:
        der["ta_busy"] = vals["TA_TA_BUSY_sum"] / (CUS * kc)
    if "TA_ADDR_STALLED_BY_TC_CYCLES_sum" in vals:
        der["ta_stalled_by_tc"] = vals["TA_ADDR_STALLED_BY_TC_CYCLES_sum"] / (CUS * kc)
    if "TCP_PENDING_STALL_CYCLES_sum" in vals:
        der["tcp_pending_stall"] = vals["TCP_PENDING_STALL_CYCLES_sum"] / (CUS * kc)
    if "SQ_ACTIVE_INST_VALU" in vals and "SQ_INSTS_VALU" in vals:
        out["note"] = ("SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU = %.3f: the busy counter returns the instruction "
                       "count on this stack, so only issue-count fractions are derived" %
                       (vals["SQ_ACTIVE_INST_VALU"] / vals["SQ_INSTS_VALU"]))
    out["derived"] = der
print(json.dumps(out, indent=1))
