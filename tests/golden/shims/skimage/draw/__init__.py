"""Stand-in for skimage.draw (Visualizer only; never on the sampling path)."""


def disk(*args, **kwargs):
    raise NotImplementedError("skimage is not available in this container")
