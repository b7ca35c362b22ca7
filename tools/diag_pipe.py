"""Pipelined vs one-generation score kernel on small TransE cases (GPU box):
max |weight - oracle| for each, so a hazard in the pipelined kernel shows as
a case-dependent error. usage: python tools/diag_pipe.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402,F401

from tests.test_gpu_step import run_case  # noqa: E402


def main():
    from KGE import _hip, loss, score
    lib = _hip.lib()
    cases = [(16, 300, 40, 3), (16, 200, 40, 3), (16, 300, 40, 7), (16, 300, 40, 50), (16, 512, 40, 3),
             (16, 256, 40, 3), (16, 257, 40, 3), (16, 600, 8, 3)]
    for d, B, K, E in cases:
        out = []
        for flags in (0, _hip.FLAG_SCORE_CLASSIC):
            ref, got, l_, ps, ns, _, _ = run_case(lib, "TransE", d, B, K, "h+t", score.LpDistance(2),
                                                  loss.SelfAdversarialNegativeSamplingLoss(1.0, 0.5), E=E, R=2,
                                                  flags=flags)
            err = np.abs(got["ent_emb"] - ref["weights"]["ent_emb"])
            rerr = np.abs(got["rel_emb"] - ref["weights"]["rel_emb"])
            out.append((err.max(), np.unravel_index(err.argmax(), err.shape), rerr.max(), got))
        dd = np.abs(out[0][3]["ent_emb"] - out[1][3]["ent_emb"])
        print("d=%d B=%d K=%d E=%d  pipe ent %.2e at %s rel %.2e | classic ent %.2e at %s rel %.2e | pipe-classic %.2e"
              % (d, B, K, E, out[0][0], out[0][1], out[0][2], out[1][0], out[1][1], out[1][2], dd.max()), flush=True)


if __name__ == "__main__":
    main()
