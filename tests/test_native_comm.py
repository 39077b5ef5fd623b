"""The C ABI's own RCCL exchange (qe_comm_* + qe_hashagg_exchange): a world-1
communicator on one GPU (RCCL refuses two ranks on one device, so more ranks run only on a
multi-GPU node). Fixed slots, the fallback when a partition outgrows its slot, and a stream-ordered
partial exported without a host wait — each against the oracle (Main.kt:1309-1325 two-phase
aggregate, HashAggregateExec K:615-651)."""
import numpy as np
import pytest

from kquery import native as N
from kquery.aggregate import HashAggregateState
from oracle import semantics as S

from test_gpu_parity import assert_groups_equal, dcol, result_dict

pytestmark = pytest.mark.gpu

AGGS = [(N.AGG_SUM, N.TYPE_INT64), (N.AGG_COUNT_STAR, N.TYPE_INT64), (N.AGG_MIN, N.TYPE_INT64),
        (N.AGG_MAX, N.TYPE_INT64)]
FNS = [f for f, _ in AGGS]


@pytest.fixture(scope="module")
def comm(gpu_ctx):
    from kquery.exchange import NativeComm

    c = NativeComm(gpu_ctx)
    yield c
    c.close()


@pytest.mark.parametrize("slot_records,expected,async_update", [(0, 8192, False), (10, 8192, False),
                                                                (0, 8192, True), (8192, 16, True)])
def test_native_exchange_world1(gpu_ctx, comm, slot_records, expected, async_update):
    from kquery.exchange import exchange_partials_native

    rng = np.random.default_rng(slot_records + expected)
    n = 200_000
    k = rng.integers(0, 5000, n).astype(np.int64) * 3 + 1
    x = rng.integers(-1000, 1000, n).astype(np.int64)
    part = HashAggregateState(gpu_ctx, [N.TYPE_INT64], AGGS, expected, async_update=async_update)
    owner = HashAggregateState(gpu_ctx, [N.TYPE_INT64], AGGS, 8192)
    X = dcol(gpu_ctx, N.TYPE_INT64, x)
    part.update([dcol(gpu_ctx, N.TYPE_INT64, k)], [X, None, X, X])
    got = exchange_partials_native(part, owner, comm, slot_records)
    assert got == len(np.unique(k))
    kk, aa = owner.finalize()
    ref = S.group_aggregate([k], [None], [x, None, x, x], [None] * 4, FNS)
    assert_groups_equal(result_dict(kk, aa), ref, FNS)


def test_native_exchange_repeated_steps(gpu_ctx, comm):
    """bench.py --exchange --exchange-impl native: reset -> update -> exchange -> finalize, several
    times on the same states and communicator buffers."""
    from kquery.datasource import C4_COLUMNS, generate_column
    from kquery.exchange import exchange_partials_native
    from kquery.workloads import c4_spec
    from oracle import gen

    n = 1_000_003
    cols = [generate_column(s, n, 0, 42, gpu_ctx) for s in C4_COLUMNS]
    part = HashAggregateState(gpu_ctx, [N.TYPE_INT64], AGGS, 1024, async_update=True)
    owner = HashAggregateState(gpu_ctx, [N.TYPE_INT64], AGGS, 1024)
    k, _ = gen.generate(gen.GEN_MOD, 1024, 42, 0, 0, n)
    a, _ = gen.generate(gen.GEN_MOD, 1 << 20, 42, 1, 0, n)
    b, _ = gen.generate(gen.GEN_MOD, 1 << 20, 42, 2, 0, n)
    ref = S.group_aggregate([k], [None], [a + b, None, a, b], [None] * 4, FNS, a > (1 << 19))
    for _ in range(3):
        part.reset()
        owner.reset()
        part.update_fused(cols, c4_spec())
        assert exchange_partials_native(part, owner, comm) == 1024
        kk, aa = owner.finalize()
        assert_groups_equal(result_dict(kk, aa), ref, FNS)


def test_comm_rejects_bad_arguments(gpu_ctx):
    uid = (N.C.c_char * N.COMM_ID_BYTES)()
    h = N.C.c_void_p()
    assert N.lib().qe_comm_create(gpu_ctx.handle, 2, 5, uid, N.C.byref(h)) == N.QE_ERR_INVALID_ARG
    assert N.lib().qe_hashagg_exchange(None, None, None, 0, None) == N.QE_ERR_INVALID_ARG


def test_slot_capacity_ignores_the_ranks_own_groups(gpu_ctx):
    """the exchange's slot size must be the same on every rank. It comes from the
    expected groups given at create time (qe_hashagg_slot_capacity), not from the sizing hint an
    update raises once this rank's own groups outgrow the LDS table."""
    import numpy as np

    from kquery import native as N
    from kquery.aggregate import HashAggregateState
    from kquery.columnar import DeviceColumn

    st = HashAggregateState(gpu_ctx, [N.TYPE_INT64], [(N.AGG_COUNT_STAR, N.TYPE_INT64)], 1024)
    before = [st.slot_capacity(w) for w in (1, 2, 8)]
    assert before == [1024, min(1024, -(-3 * 1024 // 4) + 32), min(1024, -(-3 * 1024 // 16) + 32)]
    k = np.random.default_rng(3).integers(0, 60_000, 400_000).astype(np.int64)
    for _ in range(2):  # the second batch runs with the state adapted to ~60K groups
        st.update([DeviceColumn.from_numpy(N.TYPE_INT64, k, ctx=gpu_ctx)], [None])
    assert st.num_groups() == len(np.unique(k))
    assert [st.slot_capacity(w) for w in (1, 2, 8)] == before
