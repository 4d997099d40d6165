"""Tier T3: the gfx950 fill / verify / reduce kernels against the plain
PyTorch reference of the same op (integer PRNG + word compare + checksum)."""
import pytest
import torch

from test_nccl_p2p_amd.ops import checksum, fill_, reference_bytes, reference_verify, verify

pytestmark = pytest.mark.gpu

SIZES = [16, 48, 1000, 4096, 4099, (1 << 20) + 13, 4 << 20, 64 << 20]


@pytest.fixture(scope="module", autouse=True)
def _gpu(native):
    assert torch.cuda.is_available(), "GPU tier needs a GPU"
    torch.cuda.set_device(0)


def dev_bytes(n):
    # Over-allocate so the tail path cannot write past the logical size unnoticed.
    return torch.full((n + 64,), 0xAB, dtype=torch.uint8, device="cuda")


@pytest.mark.parametrize("nbytes", SIZES)
def test_fill_matches_reference(nbytes):
    buf = dev_bytes(nbytes)
    fill_(buf[:nbytes], 0xC0FFEE)
    torch.cuda.synchronize()
    ref = reference_bytes(nbytes, 0xC0FFEE, device="cuda")
    assert torch.equal(buf[:nbytes], ref)
    assert torch.all(buf[nbytes:] == 0xAB), "fill wrote past the end"


@pytest.mark.parametrize("coherent", [False, True])
@pytest.mark.parametrize("nbytes", [16, 48, 4096, 4099, 4096 * 3 + 1008, (1 << 20) + 13, 64 << 20])
def test_copy_kernel_matches_torch(nbytes, coherent):
    """The IPC data mover (plain, and the cross-GPU form with system-scope
    sc0 sc1 buffer loads / stores) against torch's copy_, tails included,
    and nothing written past the end."""
    from test_nccl_p2p_amd import require_native
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
    dst = dev_bytes(nbytes)
    require_native().copy(dst.data_ptr(), src.data_ptr(), nbytes, torch.cuda.current_stream().cuda_stream,
                          coherent=coherent)
    torch.cuda.synchronize()
    assert torch.equal(dst[:nbytes], src)
    assert torch.all(dst[nbytes:] == 0xAB), "copy wrote past the end"


# auto and the full grid (the one fill kernel since round 5)
@pytest.mark.parametrize("fill_impl", [0, 1])
@pytest.mark.parametrize("nbytes", SIZES + [(64 << 20) + 4])
def test_fill_variants_match_reference(fill_impl, nbytes):
    from test_nccl_p2p_amd import require_native
    buf = dev_bytes(nbytes)
    require_native().fill(buf.data_ptr(), nbytes, 0xBEEF, torch.cuda.current_stream().cuda_stream, fill_impl)
    torch.cuda.synchronize()
    assert torch.equal(buf[:nbytes], reference_bytes(nbytes, 0xBEEF, device="cuda"))
    assert torch.all(buf[nbytes:] == 0xAB), "fill wrote past the end"


@pytest.mark.parametrize("impl", ["lds8", "stride"])
@pytest.mark.parametrize("nbytes", SIZES)
def test_verify_clean_and_checksum(impl, nbytes):
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    fill_(buf, 77)
    r = verify(buf, 77, impl=impl)
    ref = reference_verify(buf, 77)
    assert r.mismatches == 0 and r.first_bad == 2**64 - 1
    assert r.checksum == ref.checksum
    assert checksum(buf, impl=impl) == ref.checksum
    wrong = verify(buf, 78, impl=impl)
    assert wrong.mismatches == reference_verify(buf, 78).mismatches > 0


@pytest.mark.parametrize("impl", ["lds8", "stride"])
def test_verify_counts_exact_bitflips(impl):
    nbytes = (8 << 20) + 5
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    fill_(buf, 1234)
    flips = [7, 4096, 123457, nbytes - 1, nbytes - 3, 5 << 20]
    for off in flips:
        buf[off] ^= 0x40
    r = verify(buf, 1234, impl=impl)
    ref = reference_verify(buf, 1234)
    words = {(o // 4) for o in flips}
    assert r.mismatches == ref.mismatches == len(words)
    assert r.first_bad == ref.first_bad == 4
    assert r.checksum == ref.checksum


def test_batched_verify_matches_reference_per_buffer(native):
    """dev::launch_multi_verify (the post-timing check of many receive slots
    in one launch per 32 buffers, one readback): every job's mismatches,
    checksum and first bad byte equal the PyTorch reference of that buffer,
    across batch boundaries (40 jobs), tails, wrong seeds and bit flips."""
    sizes = [16, 4099, 48, (1 << 20) + 13, 4 << 20, 32 << 20] * 6 + [1000, 64 << 10, 16, 4096]
    bufs, jobs, want = [], [], []
    for k, n in enumerate(sizes):
        b = torch.empty(n, dtype=torch.uint8, device="cuda")
        fill_(b, 500 + k)
        if k % 5 == 1:
            b[n // 2] ^= 0x10
            b[n - 1] ^= 0x01
        seed = 500 + k if k % 7 != 3 else 9999  # some jobs checked against the wrong stream
        bufs.append(b)
        jobs.append((b.data_ptr(), n, seed))
    torch.cuda.synchronize()
    for b, (_, n, seed) in zip(bufs, jobs):
        want.append(reference_verify(b, seed))
    got = native.verify_many(jobs, torch.cuda.current_stream().cuda_stream)
    assert len(got) == len(jobs) == 40
    for k, ((m, c, f), ref) in enumerate(zip(got, want)):
        assert (m, c, f) == (ref.mismatches, ref.checksum, ref.first_bad), (k, sizes[k], (m, c, f), ref)
    assert sum(1 for m, _, _ in got if m) >= 10
    assert native.verify_many([], 0) == []


def test_lds_and_register_agree_on_random_data():
    g = torch.Generator(device="cuda").manual_seed(0)
    buf = torch.randint(0, 256, (3 << 20,), dtype=torch.uint8, device="cuda", generator=g)
    a = verify(buf, 5, impl="stride")
    b = verify(buf, 5, impl="lds8")
    assert a == b == reference_verify(buf, 5)


def test_removed_kernel_variants_fail_loudly(native):
    """Round 5 removed the fill / verify variants that lost their A/B: asking
    for one is an error that says so, never a silent fall-back."""
    buf = dev_bytes(4096)
    stream = torch.cuda.current_stream().cuda_stream
    for impl in (2, 3, 4, 5, 6):
        with pytest.raises(ValueError, match="removed in round 5"):
            native.fill(buf.data_ptr(), 4096, 1, stream, impl)
    for name in ("lds-cached", "lds-pipe", "lds8-span", "grid"):
        with pytest.raises(ValueError, match="removed in round 5"):
            verify(buf, 1, impl=name)
    with pytest.raises(ValueError):
        native.verify(buf.data_ptr(), 4096, 1, 7, True, stream)


def test_int32_tensor_and_alignment_checks():
    t = torch.empty(1 << 16, dtype=torch.int32, device="cuda")
    fill_(t, 9)
    assert verify(t, 9).ok
    with pytest.raises(ValueError):
        verify(t.view(torch.uint8)[1:17], 9)


def test_fill_verify_beyond_16gib():
    """Word indices >= 2^32 (bytes >= 16 GiB) switch the PRNG key; sized for
    the 288 GB HBM3E of an MI355X."""
    nbytes = (20 << 30) + 12
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    fill_(buf, 99)
    r = verify(buf, 99)
    assert r.mismatches == 0
    # Window across the 2^32-word boundary against the PyTorch reference.
    from test_nccl_p2p_amd.ops.buffers import reference_words

    start_word = (1 << 32) - 64
    got = buf[start_word * 4:(start_word + 128) * 4].cpu().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    assert torch.equal(got, reference_words(start_word, 128, 99))
    buf[(17 << 30) + 5] ^= 1
    r2 = verify(buf, 99)
    assert r2.mismatches == 1 and r2.first_bad == ((17 << 30) + 5) // 4 * 4
    del buf
    torch.cuda.empty_cache()
