# A/B of the step's launch forms on one GPU: HIP-graph replay vs eager launches, and the HIP runtime's
# graph knobs (bench.py lines; RCCL writes to stdout too, so the JSON is the last line starting with '{')
mkdir -p gpurun_out/eg2
run() { tag=$1; shift; timeout -k 10 200 env "$@" > gpurun_out/eg2/$tag.json 2>gpurun_out/eg2/$tag.err || return 1
  python - gpurun_out/eg2/$tag.json $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], d["ms_per_step"], d["config"]["step_form"])
PY
}
B="python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-hmm --profile-steps 0"
if [ -n "$1" ]; then run "$@"; exit $?; fi
run g128 $B --batch 128 &&
run e128 $B --batch 128 --no-graph &&
run g128_pc0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $B --batch 128 &&
run g16 $B --batch 16 &&
run e16 $B --batch 16 --no-graph &&
run gdp128 $B --batch 128 --dp-form &&
run edp128 $B --batch 128 --dp-form --no-graph &&
run gdp128_pc0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $B --batch 128 --dp-form
