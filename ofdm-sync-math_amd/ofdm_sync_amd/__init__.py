"""ofdm_sync_amd — MI355X-native OFDM preamble-sync engine (timing metrics + CFO).

Drop-in mirrors of the reference's hot-path functions, module by module:
  sync_aa.aa_detect_streaming, sc.sc_streaming_metric,
  combined_sc_min.{minn_streaming_metric, schmidl_cox_streaming_metric},
  minn.{minn_streaming_metric, minn_streaming_metric_parameterized},
  minn_rtl.{minn_rtl_streaming_metric, detect_minn_rtl}, core.estimate_cfo_from_cp,
  park.park_streaming_metric, zc_freq.compute_frequency_metric,
  zc_v2.{matched_filter_correlation, normalize_correlation, zc_streaming_detection,
         detect_zc_peaks, detect_zc_preamble}, zc (inline combiner of zc.py:106-126)
plus batched device-resident variants (``*_batched``).  All arithmetic runs in the HIP
kernels of libofdmsync.so (C ABI: include/ofdmsync.h).
"""
from . import _lib  # noqa: F401

__version__ = "0.1.0"


def library_path() -> str:
    return _lib.LIB_PATH
