# gather A/B: default kshift_fwd_k, register form, register form with non-temporal row loads
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06j
mkdir -p $O
for rep in 1 2; do
  for v in def reg nt; do
    case $v in
      def) unset LTHM_LIB_PATH; export LTHM_KSHIFT_REG=0 ;;
      reg) unset LTHM_LIB_PATH; export LTHM_KSHIFT_REG=1 ;;
      nt) export LTHM_LIB_PATH=$GRAFT_REPO_ROOT/recommendations_amd/liblthm_hip_NT.so; export LTHM_KSHIFT_REG=1 ;;
    esac
    timeout -k 10 120 python tools/gather_bench.py > $O/g_${v}_$rep.json 2> $O/g_${v}_$rep.err || { cat $O/g_${v}_$rep.err | tail; exit 1; }
    python3 -c "import json;d=json.load(open('$O/g_${v}_$rep.json'));print('$v $rep', d['spread_ids']['median_launch_ms'], d['spread_ids']['frac'], d['reference_ids']['median_launch_ms'])"
  done
done
