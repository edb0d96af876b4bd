#!/bin/bash
# Probe build of the library with an alternative k_odom.hip (not shipped): micro/<out>.so
# usage: micro/build_variant.sh path/to/k_odom_variant.hip out_name
set -e
D=$(cd $(dirname "$0")/../lidar-visual-odometry_amd/csrc && pwd)
O=$(dirname "$0")/_var_$2
mkdir -p $O
F="-std=c++17 -O3 --offload-arch=gfx950 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -w -I$D ${EXTRA:-}"
cp "$1" $D/_variant_k_odom.hip
for s in aloam_api k_scan k_grid k_lm k_map k_voxel; do /opt/rocm/bin/hipcc $F -c $D/$s.hip -o $O/$s.o & done
/opt/rocm/bin/hipcc $F -c $D/_variant_k_odom.hip -o $O/k_odom.o &
wait
rm -f $D/_variant_k_odom.hip
/opt/rocm/bin/hipcc $F -shared -o $(dirname "$0")/$2.so $O/*.o
