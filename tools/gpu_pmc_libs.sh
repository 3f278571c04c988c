#!/bin/bash
# PMC passes over the conv5 kernel (tools/micro_ratio.py) for several library builds ("-" = in-tree).
cd "$GRAFT_REPO_ROOT" || exit 1
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcl
cd /tmp && export TMPDIR=/tmp
P1="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE"
n=0
for lib in "$@"; do
  n=$((n+1))
  if [ "$lib" = "-" ]; then unset RGBD_HIP_LIB; else export RGBD_HIP_LIB="$R/$lib"; fi
  i=0
  for grp in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-include-regex conv3x3 --pmc $grp -d "$R/gpurun_out/pmcl/l${n}p$i" -o run --output-format csv -- python3 "$R/tools/micro_ratio.py" --iters 2 > "$R/gpurun_out/pmcl/l${n}p$i.log" 2>&1 || { echo "pmc $lib pass $i failed"; tail -5 "$R/gpurun_out/pmcl/l${n}p$i.log"; exit 1; }
  done
  echo "== $lib"
  python3 "$R/tools/pmc_table.py" $(find "$R/gpurun_out/pmcl" -path "*l${n}p*" -name "*counter_collection.csv")
done
