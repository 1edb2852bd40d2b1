#!/bin/bash
# Round 4 (v): debug of the one-pass unstuffing on three golden files.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ICX_DEC_DEBUG_UNSTUFF=1 ICX_LIB=$(pwd)/image-compression_amd/lib/libicx_op.so timeout -k 10 120 python scripts/dbg_unstuff.py 2>&1 | grep -v amdgpu.ids
