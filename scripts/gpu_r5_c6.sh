#!/bin/bash
set -o pipefail
./scripts/gpu_r5_hab.sh || exit 1
TAG=c6 ./scripts/gpu_r5_tree.sh
