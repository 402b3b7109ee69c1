"""python -m feature_detector_fast_amd: the reference binary's counterpart (cli.py)."""
import sys

from .cli import main

sys.exit(main())
