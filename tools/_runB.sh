cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/pmc_all.sh cornell && bash tools/pmc_all.sh sphere --scene sphere && bash tools/pmc_all.sh photon --scene photon && bash tools/pmc_all.sh photonfg --scene photon --fg 32
