"""MI355X-native RecBLR sequence encoder.

Public surface mirrors the reference repository:
  * ``RecBLR``, ``RecurrentLayer``, ``GatedRecurrentLayer``, ``FeedForward``,
    ``softplus_inverse`` (reference ``RecBLR.py``);
  * ``parallel_scan`` (reference ``parallel_scan.py``).
The compute path is hand-written HIP for gfx950 behind the C-ABI in
``include/recblr_hip.h`` (``datamining_recblr_amd/lib/libdmrecblr.so``).
"""
from ._lib import RecBLRNativeError
from .model import FeedForward, GatedRecurrentLayer, RecBLR, RecurrentLayer, softplus_inverse
from .scan import Scan, parallel_scan

__all__ = ["RecBLR", "RecurrentLayer", "GatedRecurrentLayer", "FeedForward",
           "softplus_inverse", "parallel_scan", "Scan", "RecBLRNativeError"]
__version__ = "0.1.0"
