#!/bin/bash
# PMC passes over tools/kbench.py (development): one rocprofv3 run per counter group, kernel trace
# only (never beside sys/runtime traces), each group within one pass's hardware limits (<= 8 SQ,
# 4 TCC, 4 TCP, 2 TA counters), then tools/pmc_summary.py over the passes.
#
# usage: tools/pmc.sh SET OUTDIR [kbench args...]
#   SET: mem    FETCH_SIZE / WRITE_SIZE, L2 hits and fabric requests, instruction mix
#        inst   VALU / SALU / LDS instructions per wave, waits (one pass; SKQ_DEV=1 SKQ_ABLATE=v in
#               the environment prices a phase: the deltas between values)
#        stall  issue waits, scalar / LDS pipes, instruction cache, L1 translation, texture addresser
#        lds    LDS instructions, bank and address conflicts
#        l1     L1 -> L2 read requests and their latency
#        bound  cycle counters for what binds a kernel (VALU busy cycles, waits, resident waves,
#               LDS conflicts, the texture addresser), each pass with GRBM_GUI_ACTIVE for the
#               kernel's cycles; tools/pmc_bound.py derives the fractions
# e.g. tools/pmc.sh stall gpurun_out/st --probes wide/chain --rounds 2
set -u
set_=$1 out=$2
shift 2
case "$set_" in
  mem) groups=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
               "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum"
               "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES") ;;
  inst) groups=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE") ;;
  stall) groups=("SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_LDS_IDX_ACTIVE"
                 "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_IFETCH_LEVEL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_BUSY_CYCLES SQ_WAVES"
                 "TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_THRASHING_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_SERIALIZATION_STALL_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum") ;;
  lds) groups=("SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU"
               "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY") ;;
  l1) groups=("TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum"
              "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES") ;;
  bound) groups=("SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
                 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
                 "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum SQ_WAVES GRBM_GUI_ACTIVE") ;;
  *) echo "unknown counter set $set_ (mem, inst, stall, lds, l1, bound)"; exit 2 ;;
esac
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/p$i" -o run -- python3 tools/kbench.py "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$out/p$i.log"; exit 1; }
  echo "pass $i ok: $grp"
done
python3 tools/pmc_summary.py "$out" > "$out/summary.txt" && grep -A14 "k_map1" "$out/summary.txt" | head -40
