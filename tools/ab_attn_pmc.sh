cd $GRAFT_REPO_ROOT
SWITCH=LTHM_ATTN_BWD_OLD PROG=tools/attn_probe.py FILTER=attn_bwd bash tools/pmc_ab.sh
