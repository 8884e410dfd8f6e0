"""Two ranks on the real kernels: ``bench.py --gpus 2 --same-gpu`` (bench.py
launches both rank processes itself) runs tensor-parallel and peer-shard decode
with two processes on GPU 0 - each with its own runtime, HBM arena, rings and
HIP kernels - over a gloo process group (RCCL refuses two ranks on one
device). The logits of the 2-rank job are compared against the plain fp32
PyTorch reference of the same step (llama.reference_step on a 1-rank model of
the same seed) at the 1-rank tolerance, and the greedy tokens must agree.
This is the part of the 8-GPU path one GPU can run with more than one rank:
sharded QKV / gate-up / vocab, row-parallel all-reduces, the vocab-parallel
argmax and the shard all-gathers."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B, CTX = 8, 64
ARGS = ["--model", "small", "--batch", str(B), "--context", str(CTX), "--steps", "1", "--warmup", "0", "--no-aux",
        "--weights", "ans", "--kv-format", "bf16", "--oversub", "1.5"]


def _run2(tmp_path, parallel: str, extra: tuple = ()) -> tuple[dict, torch.Tensor]:
    # the two rank processes share the GPU with this one: hand back what this
    # process's earlier tests cached first
    if torch.cuda.is_initialized():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    dump = str(tmp_path / f"logits2_{parallel}.pt")
    env = dict(os.environ, PYTHONPATH=ROOT, OGKM_UNIT_MIN_MB="0", OMP_NUM_THREADS="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--same-gpu", "--launch-timeout", "120",
           "--parallel", parallel] + ARGS + list(extra) + ["--dump-logits", dump]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=150)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads(lines[-1]), torch.load(dump)


@pytest.fixture(scope="module")
def fp32_reference():
    """fp32 logits of the bench's first decode step, from a 1-rank model of the same seed."""
    from ogkm import rt
    from ogkm._native import lib
    from ogkm.models import llama

    if lib.is_initialized():
        lib.shutdown()
    lib.config_reset()
    rt.init("hip", host_budget_mb=4096, hbm_budget={0: 2 << 30})
    try:
        cfg = llama.CONFIGS["small"]
        m = llama.TieredLlama(cfg, batch=B, context=CTX, max_new_tokens=4, oversub=1.5, device=0, seed=1234,
                              weight_format="ans", kv_format="bf16")
        g = torch.Generator(device="cpu").manual_seed(42)
        tok = torch.randint(0, cfg.vocab, (B,), generator=g)
        ref = llama.reference_step(cfg, m, tok, m.pos).float().cpu()
        m.close()
    finally:
        lib.shutdown()
        lib.config_reset()
    return ref


@pytest.mark.timeout(300)  # three processes start HIP (2 ranks + this one); the bench itself takes seconds
@pytest.mark.parametrize("parallel", ["tp", "shards", "shards-dup"])
def test_two_ranks_match_fp32_reference(fp32_reference, tmp_path, parallel):
    # shards-dup: a budget of 2.5x the rank's shard footprint - every gathered
    # unit stays on each rank as a read duplicate after its first gather
    extra = ("--oversub", "0.4") if parallel == "shards-dup" else ()
    parallel = parallel.split("-")[0]
    out, logits = _run2(tmp_path, parallel, extra)
    cfg = out["config"]
    if extra:
        assert cfg["gather_cache_gb_per_gpu"] > 0
    assert out["n_gpus"] == 2 and cfg["rccl_world"] == 2 and cfg["launcher"] == "bench.py"
    assert cfg["parallelism"] == f"{parallel}2"
    assert logits.shape == fp32_reference.shape
    d = (logits.float() - fp32_reference.float()).abs()
    print(f"{parallel}: max |diff| {d.max().item():.4f}, mean {d.mean().item():.5f} "
          f"(logits |x| mean {fp32_reference.abs().mean().item():.3f})")
    # bf16 activations between the MFMA GEMMs vs the fp32 reference: measured
    # max 0.0254 / mean 0.0043 (tp) and 0.0237 / 0.0042 (shards) on logits of
    # mean magnitude 0.51 (gpurun_out/r5/e_tp2.log)
    torch.testing.assert_close(logits, fp32_reference, atol=0.035, rtol=0.01)
    assert d.mean().item() < 0.006
    # greedy tokens: equal wherever the reference's top-2 margin exceeds the tolerance
    top2 = fp32_reference.topk(2, dim=-1).values
    clear = (top2[:, 0] - top2[:, 1]) > 0.05
    assert int(clear.sum()) >= B // 2
    assert torch.equal(logits.argmax(-1)[clear], fp32_reference.argmax(-1)[clear])
