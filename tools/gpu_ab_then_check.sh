#!/bin/bash
# One gpurun call: interleaved kernel A/B (VARS) and then the full GPU check
# (tests, smoke, bench, rocprof) of the in-tree library.  Stops at the first
# failing step.
set -o pipefail
VARS="${VARS:-base}" REPS=${REPS:-2} bash tools/ab_kernels.sh && TAG=${TAG:-run} bash tools/gpu_check.sh
