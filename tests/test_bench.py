"""bench.py's contract pieces that run without a GPU: argument defaults, the tune set the parity
test re-applies, the effective-CPU count of the CPU baseline."""
import bench


class _FakeSnap:
    program = None

    def __init__(self):
        self.tuned = {}

    def tune(self, k, v):
        self.tuned[k] = int(v)


def test_defaults_and_tune_set():
    a = bench.parse([])
    assert a.gpus == 1 and a.inflight == 4 and a.back_wgs == 3 and a.tuples == 1e9
    assert a.parity >= 1_000_000 and a.latency_batches >= 200
    s = _FakeSnap()
    bench.apply_tune(s, a)
    for k in ("stream_ecap", "stream_steal", "back_wgs", "stream_wgs", "grid_wgs", "grid_reserve"):
        assert k in s.tuned, k
    c3 = bench.parse(["--preset", "1"])
    assert c3.back_wgs == 1 and c3.grid_wgs == 4 and c3.stream_wgs == 3
    assert a.grid_wgs == 2 and a.stream_wgs == 2
    assert bench.parse(["--heavy-tail"]).tuples >= 1e8


def test_effective_cpus():
    c = bench.effective_cpus()
    assert 1 <= c["effective"] <= c["affinity"] <= c["nproc"]
