#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/ab_variants.sh noprime wd7 wd8 && bash tools/gpu_r04_full.sh
