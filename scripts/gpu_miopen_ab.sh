# Step-time A/B of MIOpen solver switches (the atomic backward-weights kernels bring SetTensor /
# CastTensor helper launches; the NHWC implicit-GEMM kernels on NCHW maps bring layout transposes).
set -o pipefail
mkdir -p gpurun_out/mab
run() {
  name=$1; shift
  env "$@" timeout -k 10 500 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pmc-traffic 0 \
      --in-graph-prof 0 > gpurun_out/mab/$name.json 2> gpurun_out/mab/$name.log || { tail -5 gpurun_out/mab/$name.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/mab/$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'])"
}
run base LSS_X=0
run nowrwgtc MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0
run nogtc MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
run base2 LSS_X=0
