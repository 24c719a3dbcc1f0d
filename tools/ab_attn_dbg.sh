cd $GRAFT_REPO_ROOT
for d in 0 1 2 3; do TAG=dbg$d LTHM_ATTN_DBG=$d LTHM_ATTN_BWD_OLD=0 timeout -k 10 120 python3 tools/attn_probe.py || exit 1; done
