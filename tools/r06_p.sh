# generator row-pass occupancy A/B (LTHM_KAG_BPC workgroups per CU)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06p
mkdir -p $O
for rep in 1 2; do
  for b in 16 32 8; do
    LTHM_KAG_BPC=$b timeout -k 10 200 python tools/embgen_bench.py > $O/b${b}_$rep.log 2>&1 || { tail -20 $O/b${b}_$rep.log; exit 1; }
    echo "bpc=$b $(grep '"fused"' $O/b${b}_$rep.log | cut -c1-90 | tr '\n' ' ')"
  done
done
