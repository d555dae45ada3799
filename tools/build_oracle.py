"""Build the C restatement of the reference scorer (oracle/tpe_score.c) in
place.  Test infrastructure: the product package never references oracle/.

    python tools/build_oracle.py [--force]
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build_oracle(force=False):
    mk = os.path.join(REPO, 'oracle', 'Makefile')
    if os.path.exists(mk):
        subprocess.check_call(['make', '-s', '-C', os.path.join(REPO, 'oracle')] +
                              (['-B'] if force else []))


if __name__ == '__main__':
    build_oracle(force='--force' in sys.argv[1:])
