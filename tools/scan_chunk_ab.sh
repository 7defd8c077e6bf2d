set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-scanab}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for v in 2048 1000 500 2048 1000 500; do
  RSC_SCAN_WGS=$v timeout -k 10 200 python bench.py --only-headline --no-cpu >> $OUT/scan_wgs_$v.jsonl 2>> $OUT/scan_ab.err
done
echo done > $OUT/done
