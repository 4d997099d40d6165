"""gfx950 buffer kernels (fill / verify / reduce) on torch tensors, plus the
plain-PyTorch reference implementations they are tested against."""

from .buffers import (  # noqa: F401
    VerifyResult,
    checksum,
    fill_,
    reference_bytes,
    reference_verify,
    reference_words,
    verify,
)
