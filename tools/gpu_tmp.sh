#!/bin/bash
set -u
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread -rf -q tests/test_leiden.py -k "edge" 2>&1 | tail -15
