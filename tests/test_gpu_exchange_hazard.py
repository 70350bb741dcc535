"""Write-while-reducing hazard of the overlapped gradient exchange, on one GPU without RCCL.

``FusedTrainStep._overlapped_tail`` (fmdiff/pipelines/train/fused.py) starts bucket b's all-reduce
asynchronously and runs the backward segments of bucket b + 1 meanwhile (reference trainer:
flow_matching_lib.py:187-192, setup_distributed training_utils.py:209-222).  That is only correct if no kernel of a
later segment reads, writes or re-zeroes a gradient range whose exchange is still in flight.  Here the collectives
are replaced by stand-ins with ProcessGroupNCCL's stream pattern -- at issue the communication stream waits on an
event recorded on the current stream; ``wait()`` makes the current stream wait on an event recorded on the
communication stream -- whose "reduce" on the side stream

  1. snapshots the bucket (the collective's read of its input),
  2. poisons the bucket with NaN and spins ~20 ms (the in-flight window), then
  3. writes back 2 x the snapshot (the collective's result at world 2 with equal ranks).

A later-segment kernel that READ an in-flight bucket would pick up NaN; one that WROTE or accumulated into it
would be overwritten by the write-back (or accumulate into NaN).  Either way the step's gradient would differ from
2 x the plain (non-overlapped) step's gradient, which is what is checked, bit for bit (x2 is exact in fp32), for
every parameter, with eager steps and with the per-bucket captured graphs, from a created stream and from the
legacy null stream.
"""
import pytest
import torch

from test_gpu_unet import _build, _load_seeded

pytestmark = pytest.mark.gpu
DEV = "cuda"
SPIN_CYCLES = 40_000_000   # ~20 ms at the shader clock: longer than any later bucket's backward segments here


class _Work:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


def _standins(comm, log):
    def allreduce_async(flat, buckets=2, group=None):
        cur = torch.cuda.current_stream()
        ev0 = torch.cuda.Event()
        ev0.record(cur)
        comm.wait_event(ev0)
        with torch.cuda.stream(comm):
            snap = flat.clone()
            flat.fill_(float("nan"))
            torch.cuda._sleep(SPIN_CYCLES)
            flat.copy_(snap * 2)
        ev1 = torch.cuda.Event()
        ev1.record(comm)
        log.append(("async", flat.numel()))
        return [_Work(ev1)]

    def allreduce(flat, buckets=4, group=None):
        flat.mul_(2)
        log.append(("sync", flat.numel()))

    return allreduce_async, allreduce


@pytest.mark.parametrize("name", ["ldct_fm_test", "ldct_fm_diffusers_b64"])
def test_overlapped_exchange_never_touches_an_inflight_bucket(golden, name, monkeypatch):
    from fmdiff.pipelines.train import fused
    T, M = golden
    meta = M[name]
    x, cond = T[f"{name}/x"].to(DEV), T[f"{name}/cond"].to(DEV)
    clean = x.clamp(0, 1)
    g = torch.Generator().manual_seed(17)
    noise = torch.randn(clean.shape, generator=g).to(DEV)
    t = torch.rand(clean.shape[0], generator=g).to(DEV)

    def grads(tr, model):
        return {k: p.grad.detach().clone() for k, p in model.named_parameters()}

    # plain step (no overlap; the world-1 exchange is a no-op)
    model = _build(meta).to(DEV)
    _load_seeded(model, meta)
    tr = fused.FusedTrainStep(model, lr=1e-3, warmup=1, overlap_allreduce=False)
    tr.step(clean, cond, noise, t)
    torch.cuda.synchronize()
    ref = grads(tr, model)

    log = []
    comm = torch.cuda.Stream()
    a_async, a_sync = _standins(comm, log)
    monkeypatch.setattr(fused, "bucketed_allreduce_async", a_async)
    monkeypatch.setattr(fused, "bucketed_allreduce", a_sync)
    for where in ("created", "null"):
        for graph in (False, True):
            model = _build(meta).to(DEV)
            _load_seeded(model, meta)
            tr = fused.FusedTrainStep(model, lr=1e-3, warmup=1, overlap_allreduce=True)
            nb = len(tr.seg_buckets)
            assert nb >= 3
            st = torch.cuda.Stream() if where == "created" else torch.cuda.default_stream()
            with torch.cuda.stream(st):
                if graph:
                    tr.capture(clean, cond, warmup_iters=1, split_collectives=True, noise=noise, t=t)
                    tr.flat.grad.zero_()
                    log.clear()
                    tr.replay()
                else:
                    log.clear()
                    tr.step(clean, cond, noise, t)
            torch.cuda.synchronize()
            # every bucket but the last went through the asynchronous stand-in, the last through the blocking one
            assert [k for k, _ in log] == ["async"] * (nb - 1) + ["sync"], log
            assert sum(n for _, n in log) == tr.flat.numel
            got = grads(tr, model)
            bad = [k for k in ref if not torch.equal(got[k], 2 * ref[k])]
            assert not bad, f"{where} stream, graph={graph}: gradients touched while in flight: {bad[:8]}"
