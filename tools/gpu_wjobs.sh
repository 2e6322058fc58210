# weight-gradient group launch time by job subset (VQHMM_WGRAD_JOBMASK, timing experiment) at cfg2 and B=128
set -o pipefail
bash tools/gpu_stage_ab.sh wj1024 1024 - VQHMM_WGRAD_JOBMASK=18 VQHMM_WGRAD_JOBMASK=45 "VQHMM_WGRAD_JOBMASK=18 VQHMM_WGRAD_BIG_CHUNKS=256" "VQHMM_WGRAD_JOBMASK=18 VQHMM_WGRAD_BIG_CHUNKS=384" &&
bash tools/gpu_stage_ab.sh wj128 128 - VQHMM_WGRAD_JOBMASK=18 VQHMM_WGRAD_JOBMASK=45
