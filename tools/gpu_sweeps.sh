# The tuning sweeps behind the step's launch-time defaults (one GPU call each; results printed as
# "label ms_per_step").  usage: bash tools/gpu_sweeps.sh wgrad|head|wmax|bwdpair|tail|pv
set -o pipefail
OUT=gpurun_out/sweeps
mkdir -p $OUT
run() {  # run LABEL BATCH ENV...
  local label=$1 b=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --batch $b --no-cpu-baseline --no-hmm --steps 400 > $OUT/run.json 2>> $OUT/err.log || exit 1
  python3 -c "import json; print('$label', json.load(open('$OUT/run.json'))['ms_per_step'])"
}
case "$1" in
  wgrad)  # big-output chunk count at cfg2, minimum rows per chunk at small batches, small-output chunks
    for c in 128 192 256 512; do run "cfg2 big_chunks=$c" 1024 VQHMM_WGRAD_BIG_CHUNKS=$c; done
    for b in 256 128; do for r in 128 192 256; do run "B=$b minrows=$r" $b VQHMM_WGRAD_MINROWS=$r; done; done
    for c in 128 256 512; do run "cfg2 small_chunks=$c" 1024 VQHMM_WGRAD_SMALL_CHUNKS=$c; done ;;
  head)   # blocks per head window by batch
    for b in 1024 512 256 128; do for n in 1 2 4; do run "B=$b nbw=$n" $b VQHMM_HEAD_NBW=$n; done; done ;;
  wmax)   # waves per workgroup cap of the conv kernels
    for b in 1024 128; do for w in 16 12 8; do run "B=$b wmax=$w" $b VQHMM_CONV_WMAX=$w; done; done ;;
  bwdpair)  # fused dec_conv1 dgrad -> enc_conv2 dgrad on / off by batch
    for b in 1024 512 128; do for r in 1000000000 0; do run "B=$b bwd_pair_rows<$r" $b VQHMM_BWD_PAIR_ROWS=$r; done; done ;;
  tail)   # one-launch backward tail and fused conv pairs on / off
    for b in 1024 128; do for t in 1 0; do run "B=$b tail_fused=$t" $b VQHMM_TAIL_FUSED=$t; run "B=$b conv_fuse=$t" $b VQHMM_CONV_FUSE=$t; done; done ;;
  pv)     # fused Prior -> Viterbi: tiles only / chain only / neither (VQHMM_PV_MODE; results then invalid)
    for m in 0 1 2 3; do VQHMM_PV_MODE=$m timeout -k 10 120 python tools/infer_bench.py > $OUT/pv$m.log 2>&1; echo "pv_mode $m"; tail -1 $OUT/pv$m.log; done ;;
  *) echo "usage: $0 wgrad|head|wmax|bwdpair|tail|pv"; exit 2 ;;
esac
