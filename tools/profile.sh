#!/bin/bash
# rocprofv3 passes for bench.py (run on the GPU box via gpurun, from the repo root).
# usage: [CFG=1|2|3|5] tools/profile.sh <tag> [pass...]   passes: trace fetch write sq lat ea tcc ta tab tas tcp tcpa mix mix2 l1 list
# (per-config PMC files must be tagged ..._cfg<N>_... for bench.py to pick them up)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}; shift || true
PASSES=${@:-trace fetch write sq}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
KREGEX=${KREGEX:-k_extend|k_shadow}  # kernels the PMC passes count
STEPS=${STEPS:-32}  # the default bench line's 32 fused passes: 4 chunks of 8 frames, as in the timed region
B="python3 $R/bench.py --no-cpu-baseline --sync-check-steps 0 --iso-steps 0 --gui-steps 0 --config ${CFG:-metric}"  # every k_extend launch of the run then carries the same fused frames
for p in $PASSES; do
  case $p in
    list)  timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true ;;
    trace) timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/trace_bench.json 2> $OUT/trace_bench.log ;;
    fetch) timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/fetch -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/fetch_bench.json 2> $OUT/fetch_bench.log ;;
    write) timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/write -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/write_bench.json 2> $OUT/write_bench.log ;;
    sq)    timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_SALU --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/sq -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/sq_bench.json 2> $OUT/sq_bench.log ;;
    lat)   timeout -k 10 240 rocprofv3 --pmc VmemLatency --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/lat -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/lat_bench.json 2> $OUT/lat_bench.log ;;
    ea)    timeout -k 10 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/ea -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/ea_bench.json 2> $OUT/ea_bench.log ;;
    ta)    timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_avr --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/ta -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/ta_bench.json 2> $OUT/ta_bench.log ;;
    tas)   timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_ADDR_STALLED_BY_TC_CYCLES_sum --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/tas -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/tas_bench.json 2> $OUT/tas_bench.log ;;
    tcp)   timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE TCP_PENDING_STALL_CYCLES_sum --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/tcp -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/tcp_bench.json 2> $OUT/tcp_bench.log ;;
    tab)   timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_max --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/tab -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/tab_bench.json 2> $OUT/tab_bench.log ;;
    tcpa)  timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/tcpa -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/tcpa_bench.json 2> $OUT/tcpa_bench.log ;;
    mix)   timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/mix -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/mix_bench.json 2> $OUT/mix_bench.log ;;
    mix2)  timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CYCLES --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/mix2 -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/mix2_bench.json 2> $OUT/mix2_bench.log ;;
    l1)    timeout -k 10 240 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/l1 -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/l1_bench.json 2> $OUT/l1_bench.log ;;
    tcc)   timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/tcc -o run -- $B --steps $STEPS --warmup $STEPS > $OUT/tcc_bench.json 2> $OUT/tcc_bench.log ;;
  esac
done
echo "profile passes done: $PASSES"
