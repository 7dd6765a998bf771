#!/bin/bash
# Two A/Bs in one call: output-array pinning (tools/r03_pin.sh), storage-order pass buckets (tools/r03_ordb.sh).
set -u
tools/r03_pin.sh && tools/r03_ordb.sh
