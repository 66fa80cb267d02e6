#!/bin/bash
# Memory type of A (SPX_A_MEM: 0 default, 1 uncached, 2 fine-grained) vs
# iteration rate at C3, eta window and explicit B^-1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for am in 0 1 2; do
  for kw in '{}' '{"window":-1}'; do
    SPX_A_MEM=$am timeout -k 10 120 python tools/itbench.py --tag "amem$am" --kw "$kw" || exit $?
  done
done
