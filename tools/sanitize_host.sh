#!/bin/bash
# Host-code sanitizer builds of libeg_hip.so and the per-element workflow harness (the device code is
# not instrumented: -fsanitize goes to the host compile only), plus a plain -O1 build (optimization-
# level dependence), into _asan/<variant>/ (git-ignored).  Build here, run on the GPU box:
#   bash tools/sanitize_host.sh build
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/sanitize_host.sh run'
# ASan and UBSan must report nothing and every array must match the port; TSan reports only races
# inside the uninstrumented ROCm runtime (its internal synchronization), none in this code.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/_asan
HIPCC=/opt/rocm/bin/hipcc
CLANG=/opt/rocm/lib/llvm/bin/clang++
FLAGS=(--offload-arch=gfx950 -std=c++17 -fPIC -fno-slp-vectorize -Wno-unused-result -Wno-pass-failed -I "$ROOT/include")
if [[ ${1:-build} == build ]]; then
  for v in asan ubsan tsan o1; do
    mkdir -p "$OUT/$v"
    case $v in
      asan) H=(-O2 -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer); C=(-fsanitize=address -fno-omit-frame-pointer) ;;
      ubsan) H=(-O2 -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined); C=(-fsanitize=undefined -fno-sanitize-recover=undefined) ;;
      tsan) H=(-O3 -Xarch_host -fsanitize=thread); C=(-fsanitize=thread) ;;
      o1) H=(-O1); C=() ;;
    esac
    for tu in eg_capi.hip eg_pow16.hip; do
      "$HIPCC" "${FLAGS[@]}" "${H[@]}" -c -o "$OUT/$v/$tu.o" "$ROOT/electionguard-remote_amd/csrc/$tu" &
    done
    wait
    LH=()
    [[ ${#C[@]} -gt 0 ]] && LH=(-Xarch_host "${C[0]}")
    "$HIPCC" --offload-arch=gfx950 -shared -fPIC "${LH[@]}" -o "$OUT/$v/libeg_hip.so" "$OUT/$v"/eg_capi.hip.o "$OUT/$v"/eg_pow16.hip.o
    "$CLANG" -std=c++17 -O1 -g "${C[@]}" -pthread -Wno-deprecated-declarations -I "$ROOT/include" \
      -I "$ROOT/electionguard-remote_amd/host" -o "$OUT/$v/percall_workflow" "$ROOT/tests/cpp/percall_workflow.cpp" \
      -L "$OUT/$v" -leg_hip -Wl,-rpath,'$ORIGIN' -L "$ROOT/oracle/_build" -legoracle -Wl,-rpath,'$ORIGIN/../../oracle/_build' -lcrypto
    rm -f "$OUT/$v"/*.o
  done
else
  mkdir -p "$ROOT/gpurun_out"
  export ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:verify_asan_link_order=0
  export TSAN_OPTIONS="report_signal_unsafe=0 history_size=2"
  for v in asan ubsan o1 tsan; do
    log="$ROOT/gpurun_out/sanitize_${v}.log"
    rc=0
    (cd "$OUT/$v" && timeout -k 10 300 ./percall_workflow 44 11 > "$log" 2>&1) || rc=$?
    echo "exit $rc" >> "$log"
    [[ $rc == 124 || $rc == 137 ]] && { echo "$v: timed out"; exit 1; }
    ours=$(grep 'SUMMARY' "$log" | grep -vc 'libamdhip64\|libhsa-runtime' || true)
    echo "$v: $(grep -o '"encrypt_mismatched_arrays": [0-9]*, "verify_flag_mismatches": [0-9]*, "invalid_flags": [0-9]*' "$log" || true)," \
      "sanitizer reports outside the ROCm runtime: $ours; exit $rc"
  done
fi
