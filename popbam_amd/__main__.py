"""python -m popbam_amd <cmd> [options] <in.bam> <region>  (see popbam_amd/cli.py)"""
import sys

from .cli import main

sys.exit(main())
