"""Command line drop-in for ``python fast_consensus.py`` (fast_consensus.py:414-466).

Same flags, defaults, validation messages and exit status, same output tree:
``out_partitions_t{tau}_d{delta}_np{n_p}/1..n_p`` and ``memberships_t.../0..n_p-1``
(louvain only; the directory is created for every algorithm).  Additive flags:
``--seed`` (the reference is unseeded) and ``--device``.
"""
import argparse
import os
import sys

from ._lib import FC_ALGO_LOUVAIN, FC_ALGO_LOUVAIN_NC
from .core import ALGORITHMS, OUT_OF_SCOPE, RULES, Engine, IdGraph, algo_id, labels_to_output

DEFAULT_TAU = {'louvain': 0.2, 'cnm': 0.7, 'infomap': 0.6, 'lpm': 0.8}   # :426


def check_arguments(args):
    """fast_consensus.py:73-88 -- identical messages."""
    if args.d > 1:
        print('delta is too high. Allowed values are between 0 and 1')
        return False
    if args.d < 0:
        print('delta is too low. Allowed values are between 0 and 1')
        return False
    if args.alg not in ('louvain', 'lpm', 'cnm', 'infomap', 'leiden'):
        print('Incorrect algorithm entered. run with -h for help')
        return False
    if args.t > 1 or args.t < 0:
        print('Incorrect tau. run with -h for help')
        return False
    return True


def build_parser():
    p = argparse.ArgumentParser(description='Process some integers.')
    p.add_argument('-f', metavar='filename', type=str, nargs='?', help='file with edgelist')
    p.add_argument('-np', metavar='n_p', type=int, nargs='?', default=20,
                   help='number of input partitions for the algorithm (Default value: 20)')
    p.add_argument('-t', metavar='tau', type=float, nargs='?', help='used for filtering weak edges')
    p.add_argument('-d', metavar='del', type=float, nargs='?', default=0.02,
                   help='convergence parameter (default = 0.02). Converges when less than delta proportion '
                        'of the edges are with wt = 1')
    p.add_argument('--alg', metavar='alg', type=str, nargs='?', default='louvain',
                   help='choose from \'louvain\' , \'cnm\' , \'lpm\' , \'infomap\' ')
    p.add_argument('--seed', type=int, default=None, help=argparse.SUPPRESS)
    p.add_argument('--device', type=int, default=0, help=argparse.SUPPRESS)
    # extension: the new_consensus.py fork's weight rule (:155-163), louvain only
    p.add_argument('--rule', type=str, default='fast_consensus', choices=RULES, help=argparse.SUPPRESS)
    return p


def output_dirs(args):
    suffix = 't' + str(args.t) + '_d' + str(args.d) + '_np' + str(args.np)
    return 'out_partitions_' + suffix, 'memberships_' + suffix


def write_outputs(args, output, root='.'):
    """fast_consensus.py:440-466.  output: list of dict (louvain) or set of frozensets."""
    out_dir, mem_dir = (os.path.join(root, d) for d in output_dirs(args))
    os.makedirs(out_dir, exist_ok=True)
    os.makedirs(mem_dir, exist_ok=True)
    output = list(output)
    if args.alg == 'louvain':
        for i in range(len(output)):
            with open(mem_dir + '/' + str(i), 'w') as f:
                for k, v in sorted(output[i].items()):
                    f.write(str(k + 1) + "\t" + str(v + 1) + '\n')
            part = {}
            for node, c in output[i].items():      # group_to_partition (:55-71)
                part.setdefault(c, []).append(node)
            output[i] = part.values()
    for i, partition in enumerate(output, start=1):
        with open(out_dir + '/' + str(i), 'w') as f:
            if args.alg == 'leiden':   # :463-466 rewrites the file as vertex -> cluster, 1-based
                for j, mem in enumerate(partition.membership):
                    f.write(str(j + 1) + "\t" + str(mem[0] + 1) + '\n')
                continue
            for community in partition:
                print(*community, file=f)


def main(argv=None):
    args = build_parser().parse_args(argv)
    if args.t is None:
        args.t = DEFAULT_TAU.get(args.alg, 0.2)
    if check_arguments(args) is False:
        sys.exit(0)                               # quit() -> exit status 0 (:430-432)
    g = IdGraph.from_edgelist_file(args.f)
    algo = algo_id(args.alg)
    if algo is None:
        output = None
    else:
        if args.rule == 'new_consensus' and algo == FC_ALGO_LOUVAIN:
            algo = FC_ALGO_LOUVAIN_NC
        with Engine(device=args.device, seed=args.seed) as eng:
            eng.load_graph(g.n, g.u, g.v)
            labels, _ = eng.run(algo, args.np, args.t, args.d)
        output = labels_to_output(args.alg, g.labels, labels)
    if output is None:                            # reference: TypeError on len(None)
        raise SystemExit("fast_consensus returned None")
    write_outputs(args, output)


if __name__ == "__main__":
    main()
