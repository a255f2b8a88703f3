"""Drop-in module for the reference's ``from parallel_scan import parallel_scan``."""
from datamining_recblr_amd.scan import Scan, parallel_scan  # noqa: F401
