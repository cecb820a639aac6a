"""Drop-in for the matched-filter combiner written inline in ``zc.py`` (zc.py:106-126).

The reference has no function for it (the lines sit inside ``run_simulation``); this
module names it ``combined_matched_filter``: Σ_br conv(x_br, conj(ref[::-1])) divided by
|ref|·sqrt(max(Σ_br sliding |x_br|², 0) + 1e-12), computed by ``ofs_zc_correlate``
(OFS_ZC_COMBINED).  ``build_pss_symbol`` defaults to include_cp=True as in zc.py:39-47.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from . import zc_v2 as _v2

N_FFT = 2048
CYCLIC_PREFIX = 512
PSS_LENGTH = 62          # zc.py:30
PSS_ROOT = 25            # zc.py:31
generate_zadoff_chu = _v2.generate_zadoff_chu


def build_pss_symbol(include_cp: bool = True) -> np.ndarray:
    """zc.py:39-47: this module's N_FFT / CYCLIC_PREFIX (read at call time), passed explicitly
    so zc_v2's own module globals are never touched."""
    return _v2.build_pss_symbol(include_cp=include_cp, n_fft=N_FFT, cyclic_prefix=CYCLIC_PREFIX)


def combined_matched_filter(rx_samples, pss_reference=None, *, want_mag: bool = False):
    """combined_corr of zc.py:106-126 (1-D or [branches, T] input)."""
    if pss_reference is None:
        pss_reference = build_pss_symbol(include_cp=False)
    from_numpy = not isinstance(rx_samples, torch.Tensor)
    x = np.asarray(rx_samples) if from_numpy else rx_samples
    if x.ndim == 1:
        x = x[None]
    corr, mag = _v2.correlate_batched(x[None], pss_reference, _v2.OFS_ZC_COMBINED, want_mag=want_mag)
    if from_numpy:
        c = _lib.to_host(corr[0], np.complex128)
        return (c, _lib.to_host(mag[0], np.float64)) if want_mag else c
    return (corr[0], mag[0]) if want_mag else corr[0]


def combined_matched_filter_batched(x, pss_reference=None, *, want_corr=True, want_mag=True):
    """Batched combiner over x[B, n_branch, T] -> (corr, |corr|) device tensors [B, T+N-1]."""
    if pss_reference is None:
        pss_reference = build_pss_symbol(include_cp=False)
    return _v2.correlate_batched(x, pss_reference, _v2.OFS_ZC_COMBINED, want_corr=want_corr,
                                 want_mag=want_mag)
