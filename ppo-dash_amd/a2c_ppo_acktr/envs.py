"""Environment factory stand-in for a2c_ppo_acktr/envs.py (reference
envs.py:1-274).  The reference module wraps gym/baselines vector envs, which are
outside this engine's scope; only the VecNormalize type
that utils.get_vec_normalize tests against is provided."""


class VecNormalize(object):
    """Type marker (reference envs.py:186-229 subclasses baselines' VecNormalize)."""

    def __init__(self, *args, **kwargs):
        self.training = True
        self.ob_rms = None

    def train(self):
        self.training = True

    def eval(self):
        self.training = False


def make_vec_envs(*args, **kwargs):
    raise NotImplementedError("gym/baselines environments are outside the MI355X engine's scope; "
                              "use a2c_ppo_acktr.synthetic.SyntheticVecEnv or your own vec env")
