"""Pack the reference's FB15k-237 indexed triples (data files of the reference
repo: data/fb15k_237/train_indexed/train.csv, valid_indexed/valid.csv) into
data/ so the GPU box, which has no /root/reference, can run bench.py on the
real graph (training steps, and the evaluate() leg on the validation split)."""
import numpy as np

src = "/root/reference/data/fb15k_237/train_indexed/train.csv"
X = np.loadtxt(src, dtype=np.int64, delimiter=",")
assert X.shape[1] == 3
np.savez_compressed("data/fb15k237_train.npz", triples=X.astype(np.int32),
                    n_entities=np.int64(X[:, [0, 2]].max() + 1), n_relations=np.int64(X[:, 1].max() + 1))
print(X.shape, X[:, [0, 2]].max() + 1, X[:, 1].max() + 1)
V = np.loadtxt("/root/reference/data/fb15k_237/valid_indexed/valid.csv", dtype=np.int64, delimiter=",")
assert V.shape[1] == 3 and V[:, [0, 2]].max() < X[:, [0, 2]].max() + 1 and V[:, 1].max() < X[:, 1].max() + 1
np.savez_compressed("data/fb15k237_valid.npz", triples=V.astype(np.int32))
print(V.shape)
