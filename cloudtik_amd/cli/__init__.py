"""The ``cloudtik`` command line (see cli/main.py)."""
