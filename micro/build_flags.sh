#!/bin/bash
# Probe build of the whole library with extra compile flags (not shipped): micro/<out>.so
# usage: micro/build_flags.sh out_name "-DALOAM_LF_TIMING ..."
set -e
D=$(cd $(dirname "$0")/../lidar-visual-odometry_amd/csrc && pwd)
O=$(dirname "$0")/_var_$1
mkdir -p $O
F="-std=c++17 -O3 --offload-arch=gfx950 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -w -I$D -I$D/../../include $2"
for s in $D/*.hip; do b=$(basename $s .hip); /opt/rocm/bin/hipcc $F -c $s -o $O/$b.o & done
wait
/opt/rocm/bin/hipcc $F -shared -o $(dirname "$0")/$1.so $O/*.o
rm -rf $O
