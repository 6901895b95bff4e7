#!/bin/bash
# Host-layer sanitizer runs on a GPU box (make sanitize first): the C++ host tests
# (IVerifier/SigManager/adapters/coalescing engine, threshsign mirror) under ASan+UBSan and TSan.
# The HIP runtime is not instrumented; leak checking is off (its allocations are process-lifetime).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/san
export ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:verify_asan_link_order=0:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export TSAN_OPTIONS=report_signal_unsafe=0:halt_on_error=0:second_deadlock_stack=1:suppressions=$GRAFT_REPO_ROOT/tools/tsan.supp
rc=0
for t in address thread; do
  for b in test_host test_bls_host; do
    if [ $t = thread ]; then  # TSan needs the classic address-space layout (no ASLR)
      timeout -k 10 300 setarch "$(uname -m)" -R ./tests/cpp/san/${b}_$t > gpurun_out/san/${b}_$t.log 2>&1
    else
      timeout -k 10 300 ./tests/cpp/san/${b}_$t > gpurun_out/san/${b}_$t.log 2>&1
    fi
    r=$?
    echo "$b [$t] exit $r: $(grep -c 'WARNING: ThreadSanitizer\|ERROR: AddressSanitizer\|runtime error' gpurun_out/san/${b}_$t.log) sanitizer reports"
    [ $r -eq 0 ] || rc=$r
    [ $r -eq 124 ] || [ $r -eq 137 ] && exit $r
  done
done
exit $rc
