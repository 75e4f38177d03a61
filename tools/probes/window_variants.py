"""The driver-shape headline window (20 contacts-off steps, one ackphys_rollout launch) timed with
the host clock under variants of what surrounds the launch (GPU box): median host microseconds
over repeated windows, each bracketed by torch.cuda.synchronize() on both sides as bench.py does.

    python3 tools/probes/window_variants.py
"""
import gc
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from mujoco_playground_amd.sim import BatchedAckermannSim
    dev = torch.device("cuda:0")
    sim = BatchedAckermannSim(4096, dev, seed=0, contacts=False)
    sim.reset()
    acts = sim.random_actions(20, seed=0)
    launch = sim.rollout_launcher(acts)
    stream = torch.cuda.current_stream(dev)
    for _ in range(100):
        launch()
    torch.cuda.synchronize()

    def bench_like():
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        torch.cuda.synchronize(dev)
        ev0.record(stream)
        t0 = time.perf_counter()
        launch()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    def no_events():
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        launch()
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    def one_sync_after():
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        ev0.record(stream)
        t0 = time.perf_counter()
        launch()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    def stream_sync():
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        ev0.record(stream)
        t0 = time.perf_counter()
        launch()
        ev1.record(stream)
        stream.synchronize()
        return time.perf_counter() - t0

    def event_sync():
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        ev0.record(stream)
        t0 = time.perf_counter()
        launch()
        ev1.record(stream)
        ev1.synchronize()
        return time.perf_counter() - t0

    def prelaunch_query():
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        ev0.record(stream)
        stream.query()
        t0 = time.perf_counter()
        launch()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    variants = [("bench_like", bench_like), ("no_events", no_events), ("one_sync_after", one_sync_after),
                ("stream_sync", stream_sync), ("event_sync", event_sync), ("prelaunch_query", prelaunch_query)]
    gc.disable()
    for rnd in range(2):
        for name, fn in variants:
            ts = sorted(fn() * 1e6 for _ in range(41))
            print(f"round {rnd} {name:16s} median {ts[20]:7.1f} us  p10 {ts[4]:7.1f}  p90 {ts[36]:7.1f}", flush=True)
    gc.enable()


if __name__ == "__main__":
    main()
