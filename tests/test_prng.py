"""PRNG contract: native host code == PyTorch reference == pinned vector."""
import torch

from test_nccl_p2p_amd.ops.buffers import payload_seed, reference_bytes, reference_verify, reference_words

# Known answer printed by tests/host/test_main.cpp (test_prng_fill_verify).
KAT = [0x01E47B8A, 0x40D8809D, 0xE869AF88, 0xFBB1D5F7]


def test_known_answer(native):
    assert [native.prng_word(0x1234, i) for i in range(4)] == KAT
    assert reference_words(0, 4, 0x1234).tolist() == KAT


def test_high_word_indices(native):
    for idx in [(1 << 32) - 1, 1 << 32, (1 << 33) + 17]:
        assert native.prng_word(99, idx) == reference_words(idx, 1, 99).item()


def test_bytes_and_verify_roundtrip(native):
    for nbytes in [1, 2, 3, 5, 16, 4099, 1 << 16]:
        hb = native.host_fill(nbytes, 7)
        rb = reference_bytes(nbytes, 7)
        assert bytes(rb.tolist()) == hb
        assert tuple(native.host_verify(hb, 7)) == tuple(reference_verify(rb, 7))


def test_corruption_counted(native):
    rb = reference_bytes(4096, 5).clone()
    rb[100] ^= 1
    rb[3000] ^= 0x80
    r = reference_verify(rb, 5)
    assert r.mismatches == 2 and r.first_bad == 100
    assert tuple(native.host_verify(bytes(rb.tolist()), 5)) == tuple(r)


def test_payload_seed(native):
    for src, nb, salt in [(0, 4096, 0), (7, 1 << 30, 3), (3, 33554432, 12345)]:
        assert native.payload_seed(src, nb, salt) == payload_seed(src, nb, salt)
    assert len({payload_seed(s, 4096) for s in range(8)}) == 8
