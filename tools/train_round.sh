# Training-step times of config 3 (fp32) and config 5 (bf16) on the final tree: the reference loop body and
# train.train_step + train.Adam (tools/train_probe.py), plus the A/B of the dense kernels' cache policy.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/train_round.txt
: > $out
for args in "20" "20 --fused --our-adam" "20 --bf16 --dims=128,256,256,256" "20 --bf16 --dims=128,256,256,256 --fused --our-adam"; do
  echo "== $args" >> $out
  timeout -k 10 200 python tools/train_probe.py $args >> $out 2>&1 || exit 1
done
echo "== 20 --fused --our-adam, PG_FLAG_DENSE_A_CACHED" >> $out
PG_SPMM_FLAGS=0x1000 timeout -k 10 200 python tools/train_probe.py 20 --fused --our-adam >> $out 2>&1 || exit 1
