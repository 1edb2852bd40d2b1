#!/bin/bash
# Build a libicx variant with tuning macros (ICX_PRE, ICX_SLOT_WORDS, ICX_FDCT_TILES): build_variant.sh NAME "-DFLAG=..." -> image-compression_amd/lib/libicx_NAME.so
# KSRC=path: the kernels source to build instead of csrc/icx_kernels.hip (e.g. a git revision's, for an A/B)
set -e
cd "$(dirname "$0")/../image-compression_amd"
mkdir -p build/var lib
F="-O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -Wno-unused-value $2"
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -I csrc -c ${KSRC:-csrc/icx_kernels.hip} -o build/var/k_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -x hip -c csrc/icx_runtime.cpp -o build/var/r_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c csrc/icx_decode.hip -o build/var/d_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -x hip -c csrc/icx_decode.cpp -o build/var/dh_$1.o
g++ -O2 -std=c++17 -fPIC $2 -c csrc/icx_jpeg_parse.cpp -o build/var/p_$1.o
g++ -O2 -std=c++17 -fPIC $2 -c csrc/icx_progressive.cpp -o build/var/pg_$1.o
g++ -O2 -std=c++17 -fPIC $2 -c csrc/icx_seqdecode.cpp -o build/var/sq_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -x hip -c csrc/icx_png.cpp -o build/var/png_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -x hip -c csrc/icx_pool.cpp -o build/var/pool_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -x hip -c csrc/icx_io.cpp -o build/var/io_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/libicx_$1.so build/var/k_$1.o build/var/r_$1.o \
    build/var/d_$1.o build/var/dh_$1.o build/var/p_$1.o build/var/pg_$1.o build/var/sq_$1.o build/var/png_$1.o build/var/pool_$1.o build/var/io_$1.o -lz
