# round 5: does a HIP runtime setting remove the ~9 us compute-queue bubble after a kernel with a cross-queue edge
# (bench/xq_probe.py, graph mode)?
set -u
mkdir -p gpurun_out/xq
run() {
  echo "== $*"
  env "$@" timeout -k 10 60 python bench/xq_probe.py --us 20 --side-us 10 --arms serial,fork_only,tbo --modes graph || return 1
}
run X=0 &&
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 &&
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 &&
run DEBUG_HIP_FORCE_GRAPH_QUEUES=1 &&
run DEBUG_HIP_FORCE_GRAPH_QUEUES=2 &&
run DEBUG_HIP_FORCE_GRAPH_QUEUES=4 &&
run GPU_STREAMOPS_CP_WAIT=1 &&
run AMD_DIRECT_DISPATCH=0 &&
run GPU_NUM_MEM_DEPENDENCY=0 &&
run DEBUG_HIP_GRAPH_BATCH_SIZE=1
