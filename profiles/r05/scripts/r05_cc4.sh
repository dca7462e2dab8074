#!/bin/bash
# GPU box, round 5: the whole GPU suite and smoke after the shape-grid refinement (per-cell
# support culling of the K1 / K3 / K6 shape lists); K1 time with and without the refinement;
# K1 wave-cycle split (SQ) and instruction mix of the refined build; k_cells with 16-B stores
# (plain vs streaming) and its trace / write bytes.
cd "$GRAFT_REPO_ROOT"
o=r05/cc4
mkdir -p gpurun_out/$o
export TMPDIR=/tmp
k1="tools/probe_k1.py --cases cfg3,canonical,regions,obstacles,empty"
sq="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
mix="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
tools/gpu_session.sh \
  "600|$o/suite|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "300|$o/smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "240|$o/cells|python -u bench.py --cells --cpu-seconds 5" \
  "120|$o/cells_nt|UAM_LIB_PATH=build/variants/libuampath_cells_nt.so python -u bench.py --no-cpu-baseline --cells" \
  "300|$o/prof_cells|PASSES='trace write' bash tools/profile_bench.sh gpurun_out/$o/cellsp --cells --steps 5 --warmup 1" \
  "200|$o/k1|python -u $k1" \
  "200|$o/k1_norefine|UAM_LIB_PATH=build/variants/libuampath_norefine.so python -u $k1" \
  "120|$o/k1_sq|rocprofv3 --pmc $sq -d gpurun_out/$o/k1sq -o run --output-format csv -- python3 tools/probe_k1.py --cases cfg3 --reps 3" \
  "120|$o/k1_mix|rocprofv3 --pmc $mix -d gpurun_out/$o/k1mix -o run --output-format csv -- python3 tools/probe_k1.py --cases cfg3 --reps 3" \
  "120|$o/k1_sq_nr|UAM_LIB_PATH=build/variants/libuampath_norefine.so rocprofv3 --pmc $sq -d gpurun_out/$o/k1sqnr -o run --output-format csv -- python3 tools/probe_k1.py --cases cfg3 --reps 3"
