#!/bin/bash
# Host-only AddressSanitizer + UndefinedBehaviorSanitizer build of the JNI shim's argument
# marshalling (native/jni/srml_jni.cpp driven by native/tests/jni_shim_test.cpp through the test
# JNIEnv) and of the C-ABI validation (ops/csrc/capi_check.h, native/tests/capi_check_test.cpp),
# linked against the host stub of the srml_capi_* entry points (no GPU, no GPU sanitizer).
set -euo pipefail
cd "$(dirname "$0")/../.."
OUT=${SRML_SANITIZE_OUT:-${TMPDIR:-/tmp}/srml_sanitize}
mkdir -p "$OUT"
CXX=${CXX:-g++}
FLAGS="-std=c++17 -g -O1 -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all"
INC="-I native/include -I native/tests/jni_harness -I spark_rapids_ml_nai_amd/ops/csrc"
$CXX $FLAGS $INC native/tests/jni_shim_test.cpp native/jni/srml_jni.cpp native/tests/capi_host_stub.cpp \
  -o "$OUT/jni_shim_asan"
$CXX $FLAGS $INC native/tests/capi_check_test.cpp native/tests/capi_host_stub.cpp -o "$OUT/capi_check_asan"
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
"$OUT/jni_shim_asan"
"$OUT/capi_check_asan"
