#!/bin/bash
# build_ref_sed.sh -- TEST INFRASTRUCTURE: a second build of the reference
# shim by SURVEY.md 8(c)'s minimal recipe, to pin the forced-include prelude
# (ref_prelude.hpp, which defines `constexpr` away for the whole translation
# unit) used by libref_v3/v4.so:
#   1. copy /root/reference to a temporary directory OUTSIDE the repository,
#   2. make the two `constexpr LifeState corona =` lines (LifeAPI.hpp:1185,
#      1190) `const` there -- the only change, shown by the diff below,
#   3. compile ref_shim.cpp against that copy with no prelude,
#   4. delete the copy.
# Output: _ref/libref_sed.so.  tests/test_oracle.py::test_prelude_build_matches_minimal_recipe
# checks that both builds agree on every fixture input.
set -euo pipefail
cd "$(dirname "$0")"
REF=${REF:-/root/reference}
CXX=${CXX_REF:-/opt/rocm/lib/llvm/bin/clang++}
mkdir -p _ref
T=$(mktemp -d /tmp/lifeapi_refsed.XXXXXX)
trap 'rm -rf "$T"' EXIT
cp -r "$REF"/. "$T"/
sed -i 's/constexpr LifeState corona =/const LifeState corona =/' "$T/LifeAPI.hpp"
# exactly the two lines change
test "$(diff "$REF/LifeAPI.hpp" "$T/LifeAPI.hpp" | grep -c '^>')" -eq 2
"$CXX" -std=c++20 -O3 -fPIC -shared -pthread -march=x86-64-v3 -Wno-nonportable-include-path \
  -Wno-undefined-inline -I_ref/inc -I"$T" ref_shim.cpp -o _ref/libref_sed.so
