"""Optimizer specs with the tf.train names / arguments the reference's gin files
bind (dqn.gin:19-25, rainbow.gin:21-25, implicit_quantile.gin:27-30).  The agent
instantiates them over its flat parameter buffer; the update runs as one TF1-
faithful HIP kernel (dopamine_amd/csrc/learner.hip)."""
from dopamine_amd import ops


class AdamOptimizer(object):
  def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-08, **unused):
    self.kwargs = dict(learning_rate=learning_rate, beta1=beta1, beta2=beta2, epsilon=epsilon)

  def build(self, flat_params, segments=None):
    return ops.TF1Adam(flat_params, segments=segments, **self.kwargs)

  def __repr__(self):
    return 'AdamOptimizer(%r)' % self.kwargs


class RMSPropOptimizer(object):
  def __init__(self, learning_rate, decay=0.9, momentum=0.0, epsilon=1e-10, centered=False, **unused):
    self.kwargs = dict(learning_rate=learning_rate, decay=decay, momentum=momentum,
                       epsilon=epsilon, centered=centered)

  def build(self, flat_params, segments=None):
    return ops.TF1RMSProp(flat_params, **self.kwargs)

  def __repr__(self):
    return 'RMSPropOptimizer(%r)' % self.kwargs
