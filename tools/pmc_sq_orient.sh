#!/bin/bash
# SQ instruction-mix counters of the orientation kernel (orient_bench2.py sample), one rocprofv3 pass per set.
# usage: bash tools/pmc_sq_orient.sh OUTDIR GROUPS
out=${1:-gpurun_out/sqo}; n=${2:-20000}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES -d $out/p1 -o p1 --output-format csv -- python3 tools/orient_bench2.py $n > $out/p1.out 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS -d $out/p2 -o p2 --output-format csv -- python3 tools/orient_bench2.py $n > $out/p2.out 2>&1 || exit 1
KERNEL=orient_kernel python3 tools/pmc_sum.py $out/p1 $out/p2 2>&1 | tail -20
