"""CPU stand-in for rl._engine used by tests/test_host.py to run bench.py's rank launcher and
JSON line without a GPU (RLE_BENCH_STUB=<this file>).  Test infrastructure only."""

import time

RLE_TD7, RLE_TD3, RLE_SAC = 0, 1, 2


def device_count():
    return 8


def synchronize(device=None):
    pass


def make_config(algo, s, a, h, b, **kw):
    return dict(algo=algo, s=s, a=a, h=h, b=b, **kw)


def init_agent(algo, s, a, h, seed):
    return {}


def parse_plan(text):
    return dict(item.split("=") for item in filter(None, text.split(",")))


class Replay:
    def __init__(self, n, s, a, lap, device=0):
        self.device = device

    def fill_random(self, n, seed=0):
        pass


class Engine:
    def __init__(self, cfg, plan=None):
        self.cfg, self.n, self._plan = cfg, 0, dict(plan or {})

    def plan(self):
        return self._plan

    def set_param(self, *a):
        pass

    def bind(self, rep):
        pass

    def graph_stats(self):
        return 23, 13

    def launch_count(self):
        return self.n * 17

    def step_timed(self, n):
        time.sleep(1e-4 * n)
        self.n += n
        return 0.1 * n

    def step_async(self, n):
        time.sleep(1e-4 * n)
        self.n += n

    def synchronize(self):
        pass
