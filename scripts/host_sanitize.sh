# Host-side sanitizer pass over the CPU test suite (no GPU: GPU ASan is not available on this pool).
#   bash scripts/host_sanitize.sh [pytest args]     -> /tmp/dcf_san/{oracle,hip}.log
# 1. oracle/dcf_oracle.c built with gcc -fsanitize=address,undefined, the suite run with gcc's runtimes
#    preloaded (DCF_ORACLE_LIB points the ctypes front-end at that build);
# 2. the C ABI library built with hipcc, the sanitizers on its host code only (-Xarch_host), the suite
#    run with clang's ASan runtime preloaded (DCF_HIP_LIB): bincode / JSON key decoding, ABI argument
#    checks and the error paths that run without a device.
set -e
O=/tmp/dcf_san; mkdir -p $O
gcc -O1 -g -fPIC -std=c11 -fsanitize=address,undefined -fno-omit-frame-pointer -shared \
  -o $O/libdcf_oracle.so oracle/dcf_oracle.c -lpthread
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -Xarch_host -fsanitize=address \
  -Xarch_host -fsanitize=undefined -shared-libsan -I include -o $O/libdcf_hip.so dcf_amd/csrc/dcf_hip.hip
GA="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
CA=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export ASAN_OPTIONS=detect_leaks=0,halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1,print_stacktrace=1
DCF_ORACLE_LIB=$O/libdcf_oracle.so LD_PRELOAD="$GA" timeout 1200 python -m pytest tests -x -q -m "not gpu" \
  -p no:cacheprovider "$@" > $O/oracle.log 2>&1 || { tail -30 $O/oracle.log; exit 1; }
echo "oracle (gcc ASan+UBSan): $(tail -1 $O/oracle.log)"
# (test_cpp_mirror links a g++ program against the library: not with an instrumented build)
DCF_HIP_LIB=$O/libdcf_hip.so LD_PRELOAD="$CA" timeout 1200 python -m pytest tests -x -q -m "not gpu" \
  -k "not cpp_mirror" -p no:cacheprovider "$@" > $O/hip.log 2>&1 || { tail -30 $O/hip.log; exit 1; }
echo "C ABI host code (clang ASan+UBSan): $(tail -1 $O/hip.log)"
