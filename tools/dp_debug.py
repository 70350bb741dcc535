"""GPU-box diagnostic: world 1 and world 2 (gloo, one GPU) graph-replayed FusedTrainStep from a caller on the
default stream (tests/dp_worker.py), per-step gradient norms vs the eager world-2 run."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_gpu_dp as T  # noqa: E402

out = "/tmp/dp_debug"
os.makedirs(out, exist_ok=True)
for world, mode in ((2, "eager"), (1, "graph"), (1, "graph"), (1, "graph"), (2, "graph"), (2, "graph"), (2, "graph"),
                    (2, "graph_plain"), (2, "graph_plain")):
    r = T._run(world, out, mode=mode)[0]
    print(world, mode, "losses", r["losses"].tolist(), "gnorms", r["gnorms"].tolist(), "final", float(r["grad"].norm()),
          flush=True)
