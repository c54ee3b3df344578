"""One rank of the multi-rank GPU test (tests/test_a_multirank_gpu.py), started
by torch.distributed.run as a fresh process: localGraph_npz over the bundles
in argv[1] with the real HIP engine (DecisionSession), the LPT shard and the
gather of records to rank 0.  Each rank writes the TDRecord keys it ran to
argv[2]/rank<r>.txt."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    savedir, outdir = sys.argv[1], sys.argv[2]
    from svscope_amd import local_graph
    ran = []
    inner = local_graph.iter_batches

    def spy(rows, *a, **kw):
        ran.extend(local_graph.window_key(r) for r in rows)
        return inner(rows, *a, **kw)

    local_graph.iter_batches = spy
    args = argparse.Namespace(TSampleID="T1", NSampleID="N1", savedir=savedir, Continue=False, batch=8)
    local_graph.localGraph_npz(args)
    import torch.distributed as dist
    with open(os.path.join(outdir, "rank%s.txt" % os.environ["RANK"]), "w") as fh:
        fh.write("\n".join(ran))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
