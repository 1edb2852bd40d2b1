#!/bin/bash
# GPU-box helper: SQ counters for the icx kernels of one bench config, for one
# or more builds of libicx (ICX_LIBS="lib/a.so lib/b.so").  One counter group
# per rocprofv3 pass, kernel-trace only alongside.  SQ_PROG: the script to
# profile (default bench.py; e.g. scripts/bench_decode.py with its own SQ_ARGS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
TAG=${TAG:-sq}
ARGS=${SQ_ARGS:-"--images 48 --steps 1 --warmup 0 --no-cpu-baseline --profile 0 --no-cache --target 16000000"}
GROUPS_=${SQ_GROUPS:-"SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,GRBM_GUI_ACTIVE"}
mkdir -p gpurun_out/$TAG
cd /tmp
for lib in ${ICX_LIBS:-image-compression_amd/lib/libicx.so}; do
  name=$(basename $lib .so)
  g=0
  for grp in $GROUPS_; do
    g=$((g+1))
    ICX_LIB="$R/$lib" timeout -k 10 ${T_SQ:-300} rocprofv3 --pmc ${grp//,/ } --kernel-trace --output-format csv -d "$R/gpurun_out/$TAG/$name/g$g" -o run -- python3 "$R/${SQ_PROG:-bench.py}" $ARGS > "$R/gpurun_out/$TAG/$name.g$g.out" 2>&1 || { echo "sq $name g$g failed rc=$?"; tail -20 "$R/gpurun_out/$TAG/$name.g$g.out"; exit 1; }
  done
done
cd "$R"
python3 scripts/sq_summary.py gpurun_out/$TAG
