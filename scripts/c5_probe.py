"""Probe: how to run 64 agents' WRN-16-4 forward+backward on one MI355X (config c5).

Times one fp32 forward+backward of every agent (B images each) for
  loop     -- one model per agent, agents in sequence (the reference's per-agent training)
  grouped  -- all agents in one model whose convs have groups = N (agents stacked on channels)
  big      -- ONE model on N*B images (same FLOPs, shared weights): the batching upper bound
each with NCHW and channels_last.  Prints one line per case as it finishes.
"""
import argparse
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "distributed-learning_amd", "networks"))
from wide_resnet import Wide_ResNet  # noqa: E402


class GBlock(nn.Module):
    def __init__(self, N, cin, cout, stride):
        super().__init__()
        self.bn1 = nn.BatchNorm2d(N * cin)
        self.conv1 = nn.Conv2d(N * cin, N * cout, 3, padding=1, groups=N)
        self.bn2 = nn.BatchNorm2d(N * cout)
        self.conv2 = nn.Conv2d(N * cout, N * cout, 3, stride=stride, padding=1, groups=N)
        self.sc = None
        if stride != 1 or cin != cout:
            self.sc = nn.Conv2d(N * cin, N * cout, 1, stride=stride, groups=N)

    def forward(self, x):
        o = self.conv1(F.relu(self.bn1(x)))
        o = self.conv2(F.relu(self.bn2(o)))
        return o + (self.sc(x) if self.sc is not None else x)


class GWRN(nn.Module):
    def __init__(self, N, k=4, n=2, classes=10):
        super().__init__()
        st = [16, 16 * k, 32 * k, 64 * k]
        self.N = N
        self.conv1 = nn.Conv2d(N * 3, N * st[0], 3, padding=1, groups=N)
        blocks, cin = [], st[0]
        for i, s in enumerate([1, 2, 2]):
            for j in range(n):
                blocks.append(GBlock(N, cin, st[i + 1], s if j == 0 else 1))
                cin = st[i + 1]
        self.blocks = nn.Sequential(*blocks)
        self.bn = nn.BatchNorm2d(N * st[3])
        self.fc = nn.Conv1d(N * st[3], N * classes, 1, groups=N)

    def forward(self, x):
        o = self.blocks(self.conv1(x))
        o = F.avg_pool2d(F.relu(self.bn(o)), 8)
        return self.fc(o.flatten(2))


def timeit(fn, reps):
    if reps == 0:
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def heartbeat(period=20.0):
    import threading
    t0 = time.perf_counter()

    def beat():
        while True:
            time.sleep(period)
            print(f"  ... {time.perf_counter() - t0:.0f}s", flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main():
    heartbeat()
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=64)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cases", default="grouped,loop,big")
    ap.add_argument("--nchw-only", action="store_true")
    ap.add_argument("--benchmark", action="store_true")
    a = ap.parse_args()
    print(f"MIOPEN_FIND_MODE={os.environ.get('MIOPEN_FIND_MODE')} N={a.agents} B={a.batch}",
          flush=True)
    N, B = a.agents, a.batch
    torch.backends.cudnn.benchmark = a.benchmark
    dev = torch.device("cuda")
    for case in a.cases.split(","):
        for cl in (False, True) if not a.nchw_only else (False,):
            mf = torch.channels_last if cl else torch.contiguous_format
            t0 = time.perf_counter()
            if case == "big":
                m = Wide_ResNet(16, 4, 0.0, 10).to(dev).to(memory_format=mf)
                x = torch.randn(N * B, 3, 32, 32, device=dev).to(memory_format=mf)
                y = torch.randint(0, 10, (N * B,), device=dev)

                def fn():
                    m.zero_grad(set_to_none=False)
                    F.cross_entropy(m(x), y).backward()
            elif case == "grouped":
                m = GWRN(N).to(dev).to(memory_format=mf)
                x = torch.randn(B, N * 3, 32, 32, device=dev).to(memory_format=mf)
                y = torch.randint(0, 10, (B, N), device=dev)

                def fn():
                    m.zero_grad(set_to_none=False)
                    z = m(x).view(B, N, 10)
                    F.cross_entropy(z.reshape(B * N, 10), y.view(-1)).backward()
            else:
                ms = [Wide_ResNet(16, 4, 0.0, 10).to(dev).to(memory_format=mf) for _ in range(N)]
                xs = torch.randn(N, B, 3, 32, 32, device=dev)
                xs = [xs[i].contiguous(memory_format=mf) for i in range(N)]
                y = torch.randint(0, 10, (N, B), device=dev)

                def fn():
                    for i in range(N):
                        ms[i].zero_grad(set_to_none=False)
                        F.cross_entropy(ms[i](xs[i]), y[i]).backward()
            first = timeit(fn, 0)
            t = timeit(fn, a.reps)
            print(f"{case:8s} channels_last={cl!s:5s} first {first*1e3:9.1f} ms  step "
                  f"{t*1e3:8.2f} ms  ({N*B/t:8.0f} img/s)  setup {time.perf_counter()-t0:.1f}s",
                  flush=True)
            del fn
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
