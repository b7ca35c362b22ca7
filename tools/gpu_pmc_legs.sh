#!/bin/bash
# PMC passes (tools/gpu_pmc.sh groups) for several bench legs. usage: gpu_pmc_legs.sh tag leg [leg ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
TAG=$1; shift
for w in "$@"; do
  bash tools/gpu_pmc.sh "$TAG/$w" "$w" || exit 3
done
echo PMC_OK
