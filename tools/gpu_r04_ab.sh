#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_r04_b.sh && bash tools/gpu_r04_a.sh
