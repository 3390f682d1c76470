"""CPU: bench.py's step runners against a stand-in mapper that follows include/loam_core.h's queue
rules (solve_async enqueues a frame, wait finishes the oldest, pose / total_iterations report
the newest finished frame).  The pipelined runner (the default for the timed steps) must count
every frame once and record stream 0's pose after every frame, in order, as the blocking runner
does; one host thread per handle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class QueueMapper:
    def __init__(self, offset=0):
        self.given = None
        self.queue = []
        self.done = None
        self.offset = offset
        self.calls = []

    def input_device_batch_args(self, plan):
        self.given = plan[0]

    def solve_async(self):
        assert self.given is not None
        assert len(self.queue) < 2
        self.queue.append(self.given)
        self.given = None
        self.calls.append("async")

    def wait(self):
        self.done = self.queue.pop(0)
        self.calls.append("wait")

    def solve(self):
        self.solve_async()
        self.wait()

    def total_iterations(self):
        return 10 + self.done

    def pose(self, s):
        return (self.offset + self.done, s)


def test_pipelined_runner_counts_every_frame_once_in_order():
    import bench
    plan = [(k,) for k in range(12)]
    m = QueueMapper()
    poses = []
    it = bench.run_steps_pipelined(m, plan, 3, 6, poses)
    assert it == sum(10 + k for k in range(3, 9))
    assert poses == [(k, 0) for k in range(3, 9)]
    # each frame enqueued before the one in flight is waited for
    assert m.calls[:3] == ["async", "async", "wait"]
    assert m.calls.count("async") == m.calls.count("wait") == 6
    b = QueueMapper()
    bposes = []
    assert bench.run_steps(b, plan, 3, 6, bposes) == it
    assert bposes == poses


def test_run_handles_pipelined_threads():
    import bench
    plans = [[(k,) for k in range(8)] for _ in range(2)]
    ms = [QueueMapper(0), QueueMapper(100)]
    poses = []
    it = bench.run_handles(ms, plans, 2, 5, poses, pipelined=True)
    assert it == 2 * sum(10 + k for k in range(2, 7))
    assert poses == [(k, 0) for k in range(2, 7)]  # handle 0's stream 0 only
