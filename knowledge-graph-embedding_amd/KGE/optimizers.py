"""Optimizers with TF-2.5 keras semantics (``BaseModel.py:243-246,328``).

``train(optimizer=...)`` accepts ``"Adam"`` / ``"SGD"`` (keras defaults) or
these objects, mirroring ``tf.optimizers.SGD`` / ``tf.optimizers.Adam``:

* SGD sparse apply = ``ResourceScatterAdd(var, idx, -lr * g)`` (duplicates summed).
* Adam (keras OptimizerV2): gradients of IndexedSlices are de-duplicated
  (summed per row); ``m <- b1*m`` and ``v <- b2*v`` over ALL rows, scatter-add of
  ``(1-b1) g`` / ``(1-b2) g^2``, then a dense
  ``var -= lr_t * m / (sqrt(v) + eps)`` with
  ``lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t)``.
"""


class SGD:
    def __init__(self, learning_rate=0.01):
        self.learning_rate = float(learning_rate)


class Adam:
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.learning_rate = float(learning_rate)
        self.beta_1 = float(beta_1)
        self.beta_2 = float(beta_2)
        self.epsilon = float(epsilon)
        self.iterations = 0
        self.slots = {}


def get(optimizer):
    if isinstance(optimizer, str):
        name = optimizer.lower()
        if name == "adam":
            return Adam()
        if name == "sgd":
            return SGD()
        raise ValueError("unknown optimizer %r" % optimizer)
    if isinstance(optimizer, (SGD, Adam)):
        return optimizer
    raise ValueError("optimizer must be 'Adam', 'SGD', KGE.optimizers.SGD or KGE.optimizers.Adam")
