set -e
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --mode analytic --steps 2 --warmup 1"
timeout -k 10 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES -d gpurun_out/k3bc/p1 -o run --output-format csv -- $B > gpurun_out/k3bc_p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_IFETCH SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/k3bc/p2 -o run --output-format csv -- $B > gpurun_out/k3bc_p2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU -d gpurun_out/k3bc/p3 -o run --output-format csv -- $B > gpurun_out/k3bc_p3.log 2>&1
