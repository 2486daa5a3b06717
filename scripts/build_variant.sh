#!/bin/bash
# An A/B build of the library: the in-tree objects, with the listed kernel TUs recompiled under extra defines,
# linked as ab/libpfmpe_<name>.so (bench.py / tests load it through PFMPE_LIB_OVERRIDE).
#   scripts/build_variant.sh <name> "<-DFOO=1 ...>" [TU ...]   (TU default: pfmpe_k_f32_philox)
set -e
cd "$(dirname "$0")/.."
name=$1; defs=$2; shift 2
tus=${*:-pfmpe_k_f32_philox}
P=pf_monocular_pose_estimator_amd
(cd $P && make -s -j8 >/dev/null)
mkdir -p ab /tmp/var_$name
objs=""
for o in $P/build/*.o; do
  b=$(basename $o .o)
  if [[ " $tus " == *" $b "* ]]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function $defs \
      -c -o /tmp/var_$name/$b.o $P/csrc/$b.hip &
    objs="$objs /tmp/var_$name/$b.o"
  else
    objs="$objs $o"
  fi
done
wait
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o ab/libpfmpe_$name.so $objs
echo ab/libpfmpe_$name.so
