# per-rank compute of the 1/2/4/8-GPU c2 layouts (tools/rank_proxy.py): ep1 x 10000 rows,
# ep2 x 10000, ep4 x 10000, ep4 x 5000 (8 GPUs = 2 row groups of EP4)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-rankscale}
mkdir -p $OUT
for a in "1 10000" "2 10000" "4 10000" "4 5000"; do
  timeout -k 10 200 python -u tools/rank_proxy.py $a 2>&1 | grep -v amdgpu.ids >> $OUT/scale.txt || exit 1
done
cat $OUT/scale.txt
