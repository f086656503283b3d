#!/bin/bash
# Diagnostic / experimental variants of libcapk.so (never loaded unless CAPK_LIB_PATH names them):
#   libcapk_diag_<name>.so = the library with gemm8q.hip compiled with -DCAPK_DIAG_<NAME>;
#   a name "exp_a+b" defines CAPK_EXP_A and CAPK_EXP_B instead (library libcapk_diag_exp_a+b.so)
set -e
cd "$(dirname "$0")/../image-captioning-ml-project_amd/csrc"
make -j8 >/dev/null
for d in "$@"; do
  if [[ $d == exp_* ]]; then
    defs=""
    for x in $(echo ${d#exp_} | tr '+' ' '); do defs="$defs -DCAPK_EXP_$(echo $x | tr a-z A-Z)"; done
  else
    defs="-DCAPK_DIAG_$(echo $d | tr a-z A-Z)"
  fi
  mkdir -p build_diag
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $defs -c gemm8q.hip -o build_diag/gemm8q_$d.o
  objs=$(ls build/*.o | grep -v gemm8q.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../capk/libcapk_diag_$d.so $objs build_diag/gemm8q_$d.o -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined
  echo built ../capk/libcapk_diag_$d.so
done
