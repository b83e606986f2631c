# Build dcf_amd/libdcf_hip_<name>.so with extra -D flags (kernel-variant A/Bs):
#   bash scripts/build_variant.sh <name> -DKNOB=value ...
N=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include "$@" \
  -o dcf_amd/libdcf_hip_$N.so dcf_amd/csrc/dcf_hip.hip
