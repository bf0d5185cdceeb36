"""A2C / ACKTR updaters (reference algo/a2c_acktr.py, kfac.py) are not part of
the PPO hot path this engine implements; the name is
kept so `from a2c_ppo_acktr import algo` resolves."""


class A2C_ACKTR(object):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("A2C/ACKTR are outside the MI355X engine's scope; use algo.PPO")
