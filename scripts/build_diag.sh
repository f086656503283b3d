#!/bin/bash
# Diagnostic variants of libcapk.so (never loaded unless CAPK_LIB_PATH names them):
#   libcapk_diag_<name>.so = the library with gemm8q.hip compiled with -DCAPK_DIAG_<NAME>
set -e
cd "$(dirname "$0")/../image-captioning-ml-project_amd/csrc"
make -j8 >/dev/null
for d in "$@"; do
  U=$(echo $d | tr a-z A-Z)
  mkdir -p build_diag
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DCAPK_DIAG_$U -c gemm8q.hip -o build_diag/gemm8q_$d.o
  objs=$(ls build/*.o | grep -v gemm8q.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../capk/libcapk_diag_$d.so $objs build_diag/gemm8q_$d.o -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined
  echo built ../capk/libcapk_diag_$d.so
done
