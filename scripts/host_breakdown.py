"""Per-step host-time breakdown of the identity7 (default) or tip7 (--tip7)
engine loop (wall time of the main engine methods; --noop replaces the
kernels by no-ops to isolate Python).

    SIZE=1024 python scripts/host_breakdown.py [--noop] [--tip7]
"""
import os, sys, time, datetime as dt, collections, functools
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np, torch
from kafka_inferenceengine_amd.ops import kernels as K
E = K.ext()
NOOP = {"analysis", "reduce_partials", "gain", "propagate", "unpack", "gather", "obs_order"}
class Fake:
    def __getattr__(self, nm):
        if nm in NOOP:
            return lambda *a, **k: 0 if nm in ("analysis", "gain") else None
        return getattr(E, nm)
if "--noop" in sys.argv:      # host-only: kernels replaced by no-ops (CPU)
    f = Fake(); K.ext = lambda: f
import kafka_inferenceengine_amd as k
import kafka_inferenceengine_amd.engine.linear_kf as L
import kafka_inferenceengine_amd.engine.state as S
acc = collections.Counter(); cnt = collections.Counter(); mx = collections.Counter()
def wrap(obj, name, label=None):
    fn = getattr(obj, name); label = label or name
    @functools.wraps(fn)
    def w(*a, **kw):
        t = time.perf_counter()
        try: return fn(*a, **kw)
        finally:
            dt_ = time.perf_counter() - t
            acc[label] += dt_; cnt[label] += 1; mx[label] = max(mx[label], dt_)
    setattr(obj, name, w)
for nm in ["advance_state", "_device_bands", "_prepare_date", "do_all_bands_state", "_dump", "_assimilate_dates"]:
    wrap(L.LinearKalman, nm)
wrap(K, "analysis", "K.analysis"); wrap(K, "reduce_partials", "K.reduce"); wrap(S.LazyForecast, "handle")
import kafka_inferenceengine_amd.engine.linear_kf as LL
LL.K = K
from kafka_inferenceengine_amd.inference import iterate_time_grid
SIZE = int(os.environ.get("SIZE", "1024" if torch.cuda.is_available() else "32"))
DEV = "cuda" if torch.cuda.is_available() else "cpu"
mask = np.ones((SIZE, SIZE), bool)
TIP = "--tip7" in sys.argv
NSTEP = int(os.environ.get("NSTEP", "400" if not TIP else "60"))
dates = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(NSTEP)]
if TIP:
    obs = k.SyntheticBHRObservations(mask, dates=dates, device=DEV, n_pool=3, stream=True, cloud_fraction=0.2,
                                     n_train=500)
    fac = k.create_nonlinear_observation_operator
else:
    obs = k.SyntheticIdentityObservations(mask, dates=dates, device=DEV, n_pool=3, stream=True, cloud_fraction=0.2)
    fac = k.create_linear_observation_operator
kf = k.LinearKalman(obs, k.DeviceOutput(k.TIP_PARAMETERS), mask, fac,
                    k.TIP_PARAMETERS, state_propagation=k.propagate_information_filter_LAI)
wrap(kf.comm, "sum_f64_async", "comm.sum_f64_async")
import kafka_inferenceengine_amd.parallel.comm as CM
for cls in [c for c in vars(CM).values() if isinstance(c, type) and hasattr(c, "result")]:
    wrap(cls, "result", f"{cls.__name__}.result (host wait)")
# host latency from the last norm read-back of a date to the next analysis launch
_last = [None]
def _mark(obj, name):
    fn = getattr(obj, name)
    @functools.wraps(fn)
    def w(*a, **kw):
        try: return fn(*a, **kw)
        finally: _last[0] = time.perf_counter()
    setattr(obj, name, w)
for cls in [c for c in vars(CM).values() if isinstance(c, type) and hasattr(c, "result")]:
    _mark(cls, "result")
_an = K.analysis
def _an_w(*a, **kw):
    if _last[0] is not None:
        acc["readback -> next analysis launch"] += time.perf_counter() - _last[0]; cnt["readback -> next analysis launch"] += 1
        _last[0] = None
    return _an(*a, **kw)
K.analysis = _an_w
kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
state = kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask))
grid = [dates[0] - dt.timedelta(days=1)] + [d + dt.timedelta(days=1) for d in dates]
steps = list(iterate_time_grid(grid, dates))
import gc
_gc = []
gc.callbacks.append(lambda phase, info: _gc.append((phase, info.get("generation"), time.perf_counter())))
step_t = []
def run(lo, hi, st):
    for i in range(lo, hi):
        t, loc, first = steps[i]
        t0_ = time.perf_counter()
        segs = torch.cuda.memory_stats().get("segment.all.allocated", 0) if DEV == "cuda" else 0
        st = kf.step(t, loc, st, advance=i > 0, all_dates=dates)
        segs2 = torch.cuda.memory_stats().get("segment.all.allocated", 0) if DEV == "cuda" else 0
        step_t.append((i, time.perf_counter() - t0_, segs2 - segs))
    return st
W = NSTEP // 20
state = run(0, W, state); acc.clear(); cnt.clear()
if DEV == "cuda":
    torch.cuda.synchronize()
M = NSTEP - 2 * W
t0 = time.perf_counter(); state = run(W, W + M, state)
if DEV == "cuda":
    torch.cuda.synchronize()
T = (time.perf_counter() - t0) / M * 1e6
print(f"step {T:.0f} us")
for k_, v in acc.most_common(): print(f"{k_:34s} {v/M*1e6:7.1f} us/step  ({cnt[k_]/M:.1f} calls, max {mx[k_]*1e6:.0f} us)")
slow = sorted(step_t, key=lambda r: -r[1])[:5]
print("slowest steps (index, ms, new allocator segments):", [(i, round(t_ * 1e3, 2), sg) for i, t_, sg in slow])
print("gc events in the timed steps:", len(_gc))
print("caches", kf.cache_stats())
