set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
BENCH_ARGS="--dtype fp32" bash scripts/pmc_final.sh s26_pmcf || exit 1
cd $GRAFT_REPO_ROOT && python3 scripts/pmc_table.py $O/s26_pmcf > $O/s26_pmcf_table.md 2>&1; cat $O/s26_pmcf_table.md | head -20
