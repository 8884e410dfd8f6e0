# Corrupt-chunk hunt (70B tp8 shard, ans weights + KV): the same diagnostic
# under several runtime variants; one log per variant under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
run() {  # name, env..., -- diag args
  local name=$1; shift
  env "$@" timeout -k 10 240 python -u tools/diag_transient.py --model llama3-70b --simulate-tp 8 --steps 2 \
    > gpurun_out/var_$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -v "amdgpu.ids\|slowest\|gc gen" gpurun_out/var_$name.log | grep "step\|CORRUPT\|zero-fill" | head -12
  return $rc
}
run base OGKM_LOG_ZERO_FILL=1 &&
run serial AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3 &&
run engine0 RT_COPY_ENGINE=0 &&
run hostwait OGKM_HOST_LEASE_WAIT=1
