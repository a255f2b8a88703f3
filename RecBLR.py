"""Drop-in module for the reference's ``from RecBLR import RecBLR`` (run.py:9).

Put this repository on PYTHONPATH (or next to run.py) and the reference's
run.py / run_with_unseen.py train the MI355X encoder unchanged."""
from datamining_recblr_amd.model import (  # noqa: F401
    FeedForward, GatedRecurrentLayer, RecBLR, RecurrentLayer, softplus_inverse)
