"""Graph replays on the legacy null stream, handed to a created stream by an event.

Round 3 saw a 2-rank FusedTrainStep driven from the legacy null stream return corrupted gradient buckets (norms of
1e16 / inf) after graph replays, and FusedTrainStep refuses that configuration since round 4 (fused.py
``_own_stream``).  The multi-rank step is: replay(s) of captured graphs on the caller's stream, then RCCL works on
RCCL's own stream ordered after them by an event.  This single-process test isolates the stream part of that chain
with no collective: a captured graph writes a known pattern into a buffer, it is replayed on the null stream, an
event recorded there is waited on by a created stream, and that stream copies the buffer out; the null stream then
waits for the copy before the next replay (the write-after-read order a caller owes: without that wait the next
replay overwrites the buffer while the side stream still reads it -- measured: replay 1's copy saw 17..21 instead of
16).  If the null-stream event could complete before the replayed kernels, the copies would see stale or partial
patterns.  Result (round 5, MI355X): every copy exact for both hand-off forms, i.e. event ordering around graph
replays on the null stream is sound; the round-3 corruption is not this.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pattern_graph(buf, adds):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):   # warm-up outside the capture
        for _ in range(adds):
            buf.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(adds):
            buf.add_(1.0)
    return g


@pytest.mark.parametrize("consumer", ["event", "wait_stream"])
def test_graph_replay_on_null_stream_then_cross_stream_copy(consumer):
    torch.cuda.set_stream(torch.cuda.default_stream())   # the legacy null stream, as a caller that sets none
    assert torch.cuda.current_stream() == torch.cuda.default_stream()
    n, adds, reps = 32 << 20, 8, 12   # 128 MiB buffer: each replay runs long enough for an early event to show
    buf = torch.zeros(n, device=DEV)
    g = _pattern_graph(buf, adds)
    buf.zero_()
    side = torch.cuda.Stream()
    outs = []
    for r in range(reps):
        g.replay()   # on the null stream
        if consumer == "event":
            ev = torch.cuda.Event()
            ev.record()   # null stream
            side.wait_event(ev)
        else:
            side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            o = torch.empty(8, device=DEV)
            # the side stream reads the whole buffer: min / max / first / last elements
            o[0], o[1] = buf.min(), buf.max()
            o[2], o[3] = buf[0], buf[-1]
            o[4:] = buf[n // 2: n // 2 + 4]
            outs.append(o)
        torch.cuda.current_stream().wait_stream(side)   # the next replay writes what the side stream reads
    torch.cuda.synchronize()
    for r, o in enumerate(outs):
        want = float(adds * (r + 1))
        got = o.cpu()
        assert torch.all(got == want), (r, want, got.tolist())
    torch.cuda.set_stream(torch.cuda.default_stream())
