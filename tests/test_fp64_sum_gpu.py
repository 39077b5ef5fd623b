"""Exact fp64 SUM / AVG of the hash aggregate on MI355X (within 1e-9 relative of the
exact sum; here: the correctly rounded exact sum, bit for bit) on adversarial groups, on every
aggregation path: the plan-specialised fused kernel (per-wave fx queue), the LDS table through
qe_hashagg_update, the generic kernel, the two-bucket (spilling) pass and the radix-partitioned
pass, in the default state and with QE_HASHAGG_DETERMINISTIC (the same accumulator).

Each group holds +2^60 in the first rows of the batch and -2^60 in the last rows (different
workgroups), unit terms and other small values between them, -0.0, and — in some groups — inputs
outside the per-workgroup LDS window ([2^-44, 2^62): 1e-30 and 3e19, which take the global
accumulator), NaN or +Inf. fp64 atomics in arrival order lose the unit terms next to 2^60 (its ulp
is 256); the exact accumulator must equal math.fsum of each group. The oracle is math.fsum over
the same rows (Python's exact, correctly rounded sum)."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _data(groups, n, seed):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, groups, n).astype(np.int64)
    x = rng.choice([1.0, 1.0, 1.0, 0.5, 0.1, -0.25, 3.0, -0.0], n)
    m = rng.random(n) < 0.2
    x[m] = rng.normal(size=int(m.sum())) * 100
    perm = rng.permutation(groups)
    k[:groups] = perm
    x[:groups] = 2.0 ** 60
    k[n - groups:] = rng.permutation(groups)
    x[n - groups:] = -(2.0 ** 60)
    # inputs outside the LDS window in a tenth of the groups, NaN / +Inf in two groups
    odd = rng.choice(np.arange(groups // 2, n - groups), size=max(8, groups // 10), replace=False)
    x[odd[0::2]] = 1e-30
    x[odd[1::2]] = 3e19
    sp = rng.choice(np.arange(groups, n - groups), size=2, replace=False)
    x[sp[0]] = np.nan
    x[sp[1]] = np.inf
    return k, x


def _expected(k, x, groups):
    order = np.argsort(k, kind="stable")
    ks, xs = k[order], x[order]
    b = np.searchsorted(ks, np.arange(groups + 1))
    out = {}
    for g in range(groups):
        v = xs[b[g]:b[g + 1]]
        if len(v) == 0:
            continue
        s = float("nan") if np.isnan(v).any() else (math.inf if np.isinf(v).any() else math.fsum(v.tolist()))
        out[g] = (s, len(v))
    return out


def _same(a, b):
    return (math.isnan(a) and math.isnan(b)) or np.float64(a).tobytes() == np.float64(b).tobytes()


@pytest.mark.parametrize("deterministic", [False, True], ids=["default", "deterministic"])
@pytest.mark.parametrize("groups,expected,path", [(1024, 1024, "lds"), (300, 64, "generic"), (4500, 4500, "two-bucket"),
                                                  (65536, 65536, "partitioned"), (6, 16, "fused")])
def test_fp64_sum_adversarial(gpu_ctx, groups, expected, path, deterministic):
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    n = max(3_000_000, groups * 40)
    k, x = _data(groups, n, groups + 17)
    want = _expected(k, x, groups)
    aggs = [(N.AGG_SUM, N.TYPE_FLOAT64), (N.AGG_AVG, N.TYPE_FLOAT64), (N.AGG_COUNT_STAR, N.TYPE_INT64)]
    if path == "generic":
        N.check(N.lib().qe_ctx_set_jit(gpu_ctx.handle, 0))
    try:
        st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], aggs, expected, deterministic=deterministic)
        kc = DeviceColumn.from_numpy(N.TYPE_INT64, k, None, ctx=gpu_ctx)
        xc = DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, None, ctx=gpu_ctx)
        if path == "fused":
            spec = N.QeFusedSpec()
            spec.mask_col = -1
            spec.nterms = 0
            spec.key_cols[0] = 0
            for j in (0, 1):
                spec.inputs[j].ntokens = 1
                spec.inputs[j].tokens[0] = N.QeToken(N.TOK_COL, 1, N.QeScalar())
            st.update_fused([kc, xc], spec)
            kind = st.last_kernel_kind()
            assert kind[0], kind
        else:
            st.update([kc], [xc, xc, None])
        keys, vals = st.finalize()
        gpu_ctx.synchronize()
    finally:
        N.check(N.lib().qe_ctx_set_jit(gpu_ctx.handle, 1))
    kv = keys[0].to_numpy()
    sv, av, cv = (v.to_numpy() for v in vals)
    assert len(kv) == len(want)
    for i in range(len(kv)):
        s, c = want[int(kv[i])]
        assert int(cv[i]) == c
        assert _same(sv[i], s), (int(kv[i]), sv[i], s)
        assert _same(av[i], s / c), (int(kv[i]), av[i], s / c)


def test_fp64_sum_finalize_errors_do_not_stick(gpu_ctx):
    """An input of 2^182 or more cannot be summed exactly: finalize reports it (never a silently
    wrong sum). The failure does not leak into the state's later calls: more updates still run,
    and after a reset the state is clean (the old ctl[6] count was never cleared)."""
    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], [(N.AGG_SUM, N.TYPE_FLOAT64)], 16)
    k = np.arange(1000, dtype=np.int64) % 7
    x = np.ones(1000)
    x[500] = 2.0 ** 200
    st.update([DeviceColumn.from_numpy(N.TYPE_INT64, k, None, ctx=gpu_ctx)],
              [DeviceColumn.from_numpy(N.TYPE_FLOAT64, x, None, ctx=gpu_ctx)])
    with pytest.raises(Exception, match="not exact to 1e-9"):
        st.finalize()
    st.update([DeviceColumn.from_numpy(N.TYPE_INT64, k, None, ctx=gpu_ctx)],
              [DeviceColumn.from_numpy(N.TYPE_FLOAT64, np.ones(1000), None, ctx=gpu_ctx)])
    st.reset()
    st.update([DeviceColumn.from_numpy(N.TYPE_INT64, k, None, ctx=gpu_ctx)],
              [DeviceColumn.from_numpy(N.TYPE_FLOAT64, np.full(1000, 0.1), None, ctx=gpu_ctx)])
    keys, vals = st.finalize()
    got = dict(zip(keys[0].to_pylist(), vals[0].to_pylist()))
    for g in range(7):
        assert got[g] == math.fsum([0.1] * int(np.sum(k == g)))


_LIMBS_CHILD = r'''
import pathlib, sys
root = pathlib.Path(sys.argv[1])
sys.path[:0] = [str(root), str(root / "query-engines_amd"), str(root / "tests")]
from kquery.columnar import Context
import test_fp64_sum_gpu as T
ctx = Context.get(0)
for groups, expected, path in [(1024, 1024, "lds"), (4500, 4500, "two-bucket"), (6, 16, "fused")]:
    for det in (False, True):
        T.test_fp64_sum_adversarial(ctx, groups, expected, path, det)
print("ok")
'''


def test_fp64_sum_limb_window():
    """The opt-in limb window (QE_FX_LIMBS=1, read once per process: a child process) on the
    adversarial groups of the LDS, two-bucket and fused paths."""
    import os
    import pathlib
    import subprocess
    import sys

    root = pathlib.Path(__file__).resolve().parents[1]
    env = dict(os.environ, QE_FX_LIMBS="1")
    r = subprocess.run([sys.executable, "-c", _LIMBS_CHILD, str(root)], cwd=str(root), env=env, capture_output=True,
                       text=True, timeout=280)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
