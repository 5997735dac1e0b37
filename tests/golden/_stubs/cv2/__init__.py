"""Placeholder so the reference's dataset modules import; any use raises."""


def __getattr__(name):
    raise ImportError("cv2 is not available in this container")
