# per-rank compute of the 8-GPU layout (tools/rank_proxy.py), alternating two builds
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-rankproxy}
mkdir -p $OUT
A=npe-pfn_amd/npe_pfn/_lib/libnpfn.so
B=${LIB_B:-tools/diaglib/libnpfn_head.so}
for r in 1 2 3; do
  for L in $A $B; do
    timeout -k 10 200 env NPFN_LIB=$L python -u tools/rank_proxy.py ${ARGS:-4 5000} 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $L) |" >> $OUT/proxy.txt || exit 1
  done
done
cat $OUT/proxy.txt
