"""Tier T3, property-based (hypothesis): the gfx950 copy, fill and verify
kernels on random shapes against the plain PyTorch reference of the same op.
The example-based tests in test_kernels_gpu.py pin chosen sizes; these draw
sizes, offsets, op counts (more than one launch's kMaxCopyOps), seeds and
corruption patterns."""
import pytest
import torch

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402

from test_nccl_p2p_amd.ops import fill_, reference_bytes, reference_verify, verify  # noqa: E402

pytestmark = pytest.mark.gpu

GPU_SETTINGS = settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
ARENA = 8 << 20


@pytest.fixture(scope="module")
def arena(native):
    assert torch.cuda.is_available(), "GPU tier needs a GPU"
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(1)
    src = torch.randint(0, 256, (ARENA,), dtype=torch.uint8, device="cuda", generator=g)
    return native, src


@st.composite
def copy_groups(draw):
    """1..40 ops of 0..256 KiB (tails included) at 16-byte aligned offsets:
    sources anywhere in the arena, destinations disjoint."""
    sizes = draw(st.lists(st.integers(0, 256 << 10), min_size=1, max_size=40))
    srcs = [draw(st.integers(0, (ARENA - s) // 16)) * 16 for s in sizes]
    gaps = draw(st.lists(st.integers(0, 8), min_size=len(sizes), max_size=len(sizes)))
    return sizes, srcs, gaps, draw(st.booleans())


@GPU_SETTINGS
@given(copy_groups())
def test_copy_many_matches_torch(arena, group):
    """copy_many (the IPC transport's group of receives: one launch per 32 ops,
    the workgroup -> op lookup, uniform and uneven op sizes, the cross-GPU
    coherent form) moves exactly the bytes torch's copy_ does and writes
    nothing else."""
    native, src = arena
    sizes, srcs, gaps, coherent = group
    dst = torch.full((ARENA + (64 << 10),), 0xAB, dtype=torch.uint8, device="cuda")
    ops, want, off = [], dst.clone(), 0
    for nb, so, gap in zip(sizes, srcs, gaps):
        off += 16 * gap
        if off + nb > dst.numel():
            break
        ops.append((dst.data_ptr() + off, src.data_ptr() + so, nb))
        want[off:off + nb] = src[so:so + nb]
        off = (off + nb + 15) // 16 * 16
    native.copy_many(ops, torch.cuda.current_stream().cuda_stream, coherent)
    torch.cuda.synchronize()
    assert torch.equal(dst, want)


@GPU_SETTINGS
@given(st.integers(1, 3 << 20), st.integers(0, (1 << 64) - 1), st.sampled_from([0, 1]))
def test_fill_matches_reference_any_size(arena, nbytes, seed, impl):
    native, _ = arena
    buf = torch.full((nbytes + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    native.fill(buf.data_ptr(), nbytes, seed, torch.cuda.current_stream().cuda_stream, impl)
    torch.cuda.synchronize()
    assert torch.equal(buf[:nbytes], reference_bytes(nbytes, seed, device="cuda"))
    assert torch.all(buf[nbytes:] == 0xAB)


@GPU_SETTINGS
@given(st.integers(16, 3 << 20), st.integers(0, (1 << 63) - 1),
       st.sampled_from(["lds8", "stride"]), st.data())
def test_verify_matches_reference_on_corruption(arena, nbytes, seed, impl, data):
    """Any set of corrupted bytes: every verify kernel reports the reference's
    mismatching-word count, first bad offset and checksum."""
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    fill_(buf, seed)
    flips = data.draw(st.lists(st.integers(0, nbytes - 1), max_size=12, unique=True))
    for off in flips:
        buf[off] ^= 0x5A
    r = verify(buf, seed, impl=impl)
    ref = reference_verify(buf, seed)
    assert r == ref
    assert r.mismatches == len({o // 4 for o in flips})
    assert r.first_bad == (4 * (min(flips) // 4) if flips else 2**64 - 1)


@GPU_SETTINGS
@given(st.lists(st.tuples(st.integers(0, 1 << 20), st.integers(0, (1 << 63) - 1), st.booleans()),
                min_size=1, max_size=40), st.data())
def test_batched_verify_matches_reference(arena, jobs, data):
    """dev::launch_multi_verify on any list of buffers (empty ones, tails,
    more than one batch of 32), some corrupted: every job's result is the
    PyTorch reference's for that buffer."""
    native, _ = arena
    bufs, args = [], []
    for nbytes, seed, corrupt in jobs:
        b = torch.empty(max(nbytes, 16), dtype=torch.uint8, device="cuda")[:nbytes]
        if nbytes:
            fill_(b, seed)
            if corrupt:
                b[data.draw(st.integers(0, nbytes - 1))] ^= 0x21
        bufs.append(b)
        args.append((b.data_ptr(), nbytes, seed))
    torch.cuda.synchronize()
    got = native.verify_many(args, torch.cuda.current_stream().cuda_stream)
    for b, (_, nbytes, seed), g in zip(bufs, args, got):
        ref = reference_verify(b, seed) if nbytes else (0, 0, 2**64 - 1)
        assert tuple(g) == tuple(ref), (nbytes, seed, g, ref)
