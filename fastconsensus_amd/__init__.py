"""fastconsensus_amd -- MI355X-native fast consensus clustering (Tandon et al., PRE 2019).

Drop-in for ytabatabaee/fastconsensus's ``fast_consensus()`` hot path (louvain + lpm):
the n_p community-detection runs and the consensus-graph update run as hand-written
HIP kernels for gfx950 behind a C-ABI (include/fastconsensus_amd.h).
"""
from ._lib import FastConsensusError  # noqa: F401
from .core import (Engine, IdGraph, check_consensus_graph, fast_consensus,  # noqa: F401
                   group_to_partition, labels_to_output)

__version__ = "0.1.0"
