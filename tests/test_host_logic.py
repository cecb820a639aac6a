"""CPU: host-side logic of the Python mirror that needs no GPU."""
import numpy as np

from ofdm_sync_amd import zc, zc_v2


def test_zc_build_pss_symbol_leaves_zc_v2_globals_alone():
    """zc.build_pss_symbol uses zc's own N_FFT / CYCLIC_PREFIX (read at call time) without
    overwriting zc_v2's module globals (a caller who re-parameterised zc_v2 keeps it)."""
    n0, cp0 = zc_v2.N_FFT, zc_v2.CYCLIC_PREFIX
    zc_v2.N_FFT, zc_v2.CYCLIC_PREFIX = 256, 16
    zc.N_FFT, zc.CYCLIC_PREFIX = 512, 64
    try:
        s = zc.build_pss_symbol(include_cp=True)
        assert s.shape == (512 + 64,)
        assert (zc_v2.N_FFT, zc_v2.CYCLIC_PREFIX) == (256, 16)
        assert zc_v2.build_pss_symbol(include_cp=True).shape == (256 + 16,)
        np.testing.assert_allclose(s[64:], zc_v2.build_pss_symbol(n_fft=512, cyclic_prefix=0))
    finally:
        zc_v2.N_FFT, zc_v2.CYCLIC_PREFIX = n0, cp0
        zc.N_FFT, zc.CYCLIC_PREFIX = 2048, 512
