# Build libgpd_<name>.so from a csrc tree: bash scripts/build_variant.sh <name> <tree with gym_pybullet_drones_routing_amd/csrc/ and include/>
set -e
P=/root/repo/gym_pybullet_drones_routing_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -mllvm -amdgpu-kernarg-preload-count=12 \
  -mllvm -amdgpu-sched-strategy=max-ilp -fPIC -shared -Wall -Wno-unused-result -I$2/include $GPD_DEFS -o $P/libgpd_$1.so $2/gym_pybullet_drones_routing_amd/csrc/gpd.hip
