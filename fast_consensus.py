#!/usr/bin/env python3
"""Drop-in entry point: ``python fast_consensus.py -f FILE [--alg louvain|lpm] [-np N] [-t TAU] [-d DELTA]``
and ``from fast_consensus import fast_consensus``.  Everything runs in fastconsensus_amd."""
from fastconsensus_amd import check_consensus_graph, fast_consensus, group_to_partition  # noqa: F401
from fastconsensus_amd.cli import check_arguments, main  # noqa: F401

if __name__ == "__main__":
    main()
