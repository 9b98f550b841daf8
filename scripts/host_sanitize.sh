#!/bin/bash
# Host-side sanitizer pass ("run ASan/UBSan on the host C++"). CPU only, this
# container; nothing here runs on a GPU box.
#
# 1. libbo_amd.so's HOST code -- every csrc/*.hip compiled as in the product build (gfx950 device
#    code unchanged) with -fsanitize=address,undefined on the host side only -- loaded through
#    BO_AMD_LIB by the CPU tests that call into it: the native Powell driver
#    (bo_powell_minimize, tests/test_powell.py), the hypervolume box decomposition (bo_hvi_boxes,
#    tests/test_hvi.py's CPU cases), the Sobol generator (bo_sobol_points, tests/test_sobol.py),
#    and the ABI exports / struct layouts (tests/test_abi.py).  Python is not sanitized, so the
#    clang ASan runtime is preloaded (leak detection off: CPython's arenas are not freed at exit).
# 2. oracle/cpu_ref.c (the C/OpenMP restatement the tests and bench's cpu_baseline use), built
#    with gcc -fsanitize=address,undefined (gcc's runtime preloaded, in a separate pytest run so
#    the two ASan runtimes never meet), exercised by tests/test_oracle_golden.py.
#
# Any ASan report aborts the run (non-zero exit); UBSan reports ("runtime error:") are counted
# from the logs and fail the script.  Usage: scripts/host_sanitize.sh [log_dir]
set -u -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-/tmp/bo_sanitize}"
mkdir -p "$OUT/obj"
HIPCC=/opt/rocm/bin/hipcc
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined"
srcs="bo_predict_d2 bo_predict_d4 bo_predict_d6 bo_predict_d8 bo_predict_s2 bo_predict_s4 bo_predict_s6
      bo_predict_s8 bo_predict bo_fit bo_lu bo_select bo_misc bo_hvi bo_powell"
pids=()
for s in $srcs; do
  $HIPCC --offload-arch=gfx950 -O1 -g -fno-omit-frame-pointer -std=c++17 -fPIC -I "$ROOT/include" $SAN \
    -c "$ROOT/bayesopt_smart_amd/csrc/$s.hip" -o "$OUT/obj/$s.o" > "$OUT/obj/$s.log" 2>&1 &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p" || { echo "compile failed"; cat "$OUT"/obj/*.log; exit 1; }; done
$HIPCC --offload-arch=gfx950 -shared -fPIC $SAN -shared-libsan "$OUT"/obj/*.o -o "$OUT/libbo_amd_san.so" \
  > "$OUT/link.log" 2>&1 || { cat "$OUT/link.log"; exit 1; }
gcc -O1 -g -fno-omit-frame-pointer -march=x86-64-v3 -fopenmp -shared -fPIC -fsanitize=address,undefined \
  "$ROOT/oracle/cpu_ref.c" -o "$OUT/libcpu_ref_san.so" -lm || exit 1

CLANG_ASAN="$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)"
GCC_ASAN="$(gcc -print-file-name=libasan.so)"
GCC_UBSAN="$(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_odr_violation=0"
export UBSAN_OPTIONS="print_stacktrace=1"
cd "$ROOT"
rc=0
echo "== libbo_amd host code, ASan + UBSan ($CLANG_ASAN)"
BO_AMD_LIB="$OUT/libbo_amd_san.so" LD_PRELOAD="$CLANG_ASAN" \
  python -m pytest -q -p no:cacheprovider -m "not gpu" tests/test_powell.py tests/test_hvi.py \
  tests/test_sobol.py tests/test_abi.py > "$OUT/bo_amd.log" 2>&1 || rc=1
tail -3 "$OUT/bo_amd.log"
echo "== oracle/cpu_ref.c, ASan + UBSan ($GCC_ASAN)"
BO_CPU_REF_LIB="$OUT/libcpu_ref_san.so" LD_PRELOAD="$GCC_ASAN $GCC_UBSAN" \
  python -m pytest -q -p no:cacheprovider -m "not gpu" tests/test_oracle_golden.py > "$OUT/cpu_ref.log" 2>&1 || rc=1
tail -3 "$OUT/cpu_ref.log"
for f in "$OUT/bo_amd.log" "$OUT/cpu_ref.log"; do
  n_ub=$(grep -c "runtime error:" "$f")
  n_as=$(grep -c "ERROR: AddressSanitizer" "$f")
  echo "$(basename "$f"): UBSan reports $n_ub, ASan reports $n_as"
  [ "$n_ub" = 0 ] && [ "$n_as" = 0 ] || rc=1
done
echo "sanitizer pass: $([ $rc = 0 ] && echo CLEAN || echo FAILED)"
exit $rc
