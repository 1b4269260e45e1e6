#!/bin/bash
# round 4 (final sources): selected GPU tests, C2 / C5 A/B against the previous commit's library
# (variants/head.so), then the rocprofv3 kernel statistics of C2 / C4 / C5 / C5 + FG
cd ${GRAFT_REPO_ROOT:-/root/repo}
bash tools/gpu_r04i.sh || exit $?
bash tools/refresh_profiles.sh stats
