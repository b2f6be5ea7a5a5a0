#!/bin/bash
# The mixed-routing gloo stall vs HIP stream -> hardware-queue mapping: side stream created
# before any model, and 8 hardware queues per process.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
PHASES=80 EXTRA_ENV="CLOUDTIK_AMD_EARLY_SIDE_STREAM=1" bash scripts/gpu_gloo_mixed.sh gloo_early || exit 1
PHASES=80 EXTRA_ENV="GPU_MAX_HW_QUEUES=8" bash scripts/gpu_gloo_mixed.sh gloo_hwq8 || exit 1
