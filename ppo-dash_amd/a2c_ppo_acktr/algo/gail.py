"""GAIL (reference algo/gail.py) is outside the PPO hot path (SURVEY.md §2.1
row 12); run.py only imports the module (--gail defaults to off)."""


class Discriminator(object):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("GAIL is outside the MI355X engine's scope")


class ExpertDataset(object):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("GAIL is outside the MI355X engine's scope")
