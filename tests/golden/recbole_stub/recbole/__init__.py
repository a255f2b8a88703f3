"""Minimal stand-in for the recbole package, used ONLY by make_golden.py so the
reference RecBLR.py (which imports recbole) can be executed in this container.
recbole==1.2.0 is not installed and there is no network."""
