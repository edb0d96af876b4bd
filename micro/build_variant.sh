#!/bin/bash
# usage: micro/build_variant.sh NAME "-DFLAG ..." -> micro/_var_NAME/libaloam_hip.so (profiling builds;
# select with ALOAM_LIB_PATH)
set -e
N=$1; X=$2
D=micro/_var_$N; mkdir -p $D
S=lidar-visual-odometry_amd/csrc
FL="-std=c++17 -O3 --offload-arch=gfx950 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -mllvm -amdgpu-atomic-optimizer-strategy=DPP $X"
pids=()
for f in $S/*.hip; do b=$(basename $f .hip); /opt/rocm/bin/hipcc $FL -c $f -o $D/$b.o & pids+=($!); done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc $FL -shared -o $D/libaloam_hip.so $D/*.o
echo built $D/libaloam_hip.so
