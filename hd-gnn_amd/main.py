# -*- coding: utf-8 -*-
"""Drop-in for the reference's main.py: the same argparse surface and the same loop over
the three glide step configurations (main.py:10-73), running hdgnn.model.graph2graph on
MI355X instead of a TF1 session.

    python hd-gnn_amd/main.py --Type train [--epoch 50 --Mini_batch 50 ...]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        hd-gnn_amd/main.py --Type train          # data parallel over N GPUs (RCCL)

The dataset loader is the reference's utils2.read_data (put its directory on
PYTHONPATH, as the reference's own main.py expects it next to itself).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _init_distributed():
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not torch.distributed.is_initialized():
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))


def _variant(argv):
    """Additions to the reference's flags (every reference flag is unchanged):
    --model N (1..4, default 2 = the reference main.py's `from model_2 import`): which
    model_N.graph2graph to run; --loader utils2|fast: the reference's read_data (default)
    or hdgnn.loader reading the same dataset files straight into the compact form."""
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument('--model', type=int, default=2, choices=(1, 2, 3, 4))
    p.add_argument('--loader', default='utils2', choices=('utils2', 'fast'))
    a, rest = p.parse_known_args(argv)
    return a.model, a.loader, rest


# the reference's per-step tables (main.py:11-15): glide steps 2, 3, 5
STEPS = [2, 3, 5]
ENTITY_NODES = [200, 250, 250]
HUNK_NODES = [74, 114, 150]
ENTITY_EDGES = [39800, 62250, 62250]
HUNK_EDGES = [5402, 12882, 22350]


def build_parser(step, entity_node, hunk_node, entity_edge, hunk_edge):
    """The reference's per-step parser (main.py:24-48): same flags, types, defaults, help."""
    parser = argparse.ArgumentParser(description='')
    parser.add_argument('--epoch', type=int, default=50, help='number of training epochs')
    parser.add_argument('--Ds', type=int, default=1, help='The State Dimention')
    parser.add_argument('--Ds_inter', type=int, default=1, help='The State Dimention of inter state')
    parser.add_argument('--Dr', type=int, default=2, help='The Relationship Dimension')
    parser.add_argument('--Dr_inter', type=int, default=2, help='The Relationship Dimension of inter state')
    parser.add_argument('--De_e', type=int, default=20, help='The Effect Dimension on entity')
    parser.add_argument('--De_er', type=int, default=20, help='The Effect Dimension on entity Relations')
    parser.add_argument('--Mini_batch', type=int, default=50, help='The training mini_batch')
    parser.add_argument('--checkpoint_dir', dest='checkpoint_dir', default='./checkpoint40/',
                        help='models are saved here')
    parser.add_argument('--Ne', type=int, default=entity_node, help='The Number of entities')
    parser.add_argument('--Nc', type=int, default=hunk_node, help='The Number of code changes')
    parser.add_argument('--Ner', type=int, default=entity_edge, help='The Number of entity Relations')
    parser.add_argument('--Ncr', type=int, default=hunk_edge, help='The Number of code change Relations')
    parser.add_argument('--Step', type=int, default=step, help='the number of commits/groups')
    parser.add_argument('--Repo', type=str, default='glide', help='the name of repository')
    parser.add_argument('--Type', dest='Type', default='train', help='train or test')
    return parser


def main(argv=None, model_cls=None):
    """model_cls: the graph2graph class to run (tests inject a recorder); default
    hdgnn.model[_N].graph2graph for --model N."""
    import importlib
    variant, loader, argv = _variant(sys.argv[1:] if argv is None else argv)
    graph2graph = model_cls or importlib.import_module(
        "hdgnn.model" + ("" if variant == 2 else "_%d" % variant)).graph2graph
    if model_cls is None:
        _init_distributed()

    for step, entity_node, hunk_node, entity_edge, hunk_edge in zip(
            STEPS, ENTITY_NODES, HUNK_NODES, ENTITY_EDGES, HUNK_EDGES):
        print(step, entity_node, hunk_node, entity_edge, hunk_edge)
        args = build_parser(step, entity_node, hunk_node, entity_edge, hunk_edge).parse_args(argv)

        if not os.path.exists(args.checkpoint_dir):
            os.makedirs(args.checkpoint_dir)
        model = graph2graph(None,
                            Ds=args.Ds,
                            Ne=args.Ne, Nc=args.Nc,
                            Ner=args.Ner, Ncr=args.Ncr,
                            Dr=args.Dr,
                            De_e=args.De_e, De_er=args.De_er,
                            Mini_batch=args.Mini_batch,
                            checkpoint_dir=args.checkpoint_dir,
                            epoch=args.epoch,
                            Ds_inter=args.Ds_inter, Dr_inter=args.Dr_inter,
                            Step=args.Step,
                            Repo=args.Repo, loader=loader)
        if args.Type == 'train':
            model.train(args)
        if args.Type == 'test':
            model.test(args)


if __name__ == '__main__':
    main()
