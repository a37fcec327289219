#!/bin/bash
# A/B variants of the sorted kernel (all four modes): scripts/ab_build_sorted.sh "name:-DFLAG=V ..." ...
# [SRC=<other source of pico_csum_k_sorted.hip>] builds picotcp_amd/ab/libpicocsum_<name>.so from the
# product's other objects (make first) and the variant's four mode objects (scripts/gpu_ab.sh A=<name>).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
make -s -j8 -C picotcp_amd/csrc
mkdir -p build/csrc/ab picotcp_amd/ab
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  rm -f build/csrc/ab/${name}_m?.o
  for m in 0 1 2 3; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Iinclude -DSORTED_MODE=$m $flags \
        -c ${SRC:-picotcp_amd/csrc/pico_csum_k_sorted.hip} -o build/csrc/ab/${name}_m$m.o &
  done
  wait
  ls build/csrc/ab/${name}_m0.o build/csrc/ab/${name}_m1.o build/csrc/ab/${name}_m2.o build/csrc/ab/${name}_m3.o > /dev/null
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o picotcp_amd/ab/libpicocsum_$name.so \
      build/csrc/pico_csum_k_raw.o build/csrc/ab/${name}_m?.o build/csrc/pico_csum_k_frag.o build/csrc/pico_csum.o \
      -Wl,--no-undefined -Wl,-soname,libpicocsum.so
  echo "picotcp_amd/ab/libpicocsum_$name.so"
done
