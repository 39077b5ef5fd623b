"""Caching device allocator (qe_runtime.hip dev_alloc / dev_free, C ABI qe_device_alloc /
qe_device_free / qe_release_cached_memory): freed blocks are reused in stream order on the same
ctx, hash-aggregate states created and destroyed back to back on two contexts (two streams) keep
giving oracle results, and releasing the cache leaves the library working."""
import numpy as np
import pytest

from oracle import semantics as S

pytestmark = pytest.mark.gpu

from kquery import native as N  # noqa: E402
from kquery.aggregate import HashAggregateState  # noqa: E402
from kquery.columnar import DeviceColumn  # noqa: E402


def _alloc(ctx, n):
    p = N.C.c_void_p()
    N.check(N.lib().qe_device_alloc(ctx.handle, n, N.C.byref(p)))
    return p.value


def test_same_stream_reuse(gpu_ctx):
    a = _alloc(gpu_ctx, 3000)
    N.check(N.lib().qe_device_free(gpu_ctx.handle, a))
    b = _alloc(gpu_ctx, 4000)  # same 4 KiB size class, same stream: the freed block comes back
    assert a == b
    N.check(N.lib().qe_device_free(gpu_ctx.handle, b))
    N.check(N.lib().qe_release_cached_memory(0))


def test_states_across_two_streams(gpu_ctx):
    import torch

    from kquery.columnar import Context

    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        other = Context.get(0)
    rng = np.random.default_rng(3)
    n = 200_000
    k = rng.integers(0, 5000, n).astype(np.int64)
    x = rng.integers(-100, 100, n).astype(np.int64)
    fns = [N.AGG_SUM, N.AGG_COUNT_STAR, N.AGG_MIN, N.AGG_MAX]
    ref = S.group_aggregate([k], [None], [x] * 4, [None] * 4, fns)
    for it in range(6):
        ctx, stream = (gpu_ctx, torch.cuda.current_stream()) if it % 2 == 0 else (other, s)
        with torch.cuda.stream(stream):
            K = DeviceColumn.from_numpy(N.TYPE_INT64, k, None, ctx=ctx)
            X = DeviceColumn.from_numpy(N.TYPE_INT64, x, None, ctx=ctx)
            st = HashAggregateState(ctx, [N.TYPE_INT64], [(f, N.TYPE_INT64) for f in fns], 5000)
            st.update([K], [X] * 4)
            kk, aa = st.finalize()
            st.close()  # blocks return to the cache while this stream may still be busy
            got = {(int(a),): [int(c[i]) for c in (v.to_numpy() for v in aa)]
                   for i, a in enumerate(kk[0].to_numpy())}
            ctx.synchronize()
        assert len(got) == len(ref)
        for key, want in ref.items():
            assert got[tuple(S.canon(v) for v in key)] == [int(w) for w in want]
    N.check(N.lib().qe_release_cached_memory(0))
