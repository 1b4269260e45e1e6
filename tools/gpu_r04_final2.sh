#!/bin/bash
# round 4 final sources: C4 and C5 PMC
cd ${GRAFT_REPO_ROOT:-/root/repo}
bash tools/pmc_all.sh sphere --scene sphere && bash tools/pmc_all.sh photon --scene photon
