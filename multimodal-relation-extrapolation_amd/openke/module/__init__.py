from .BaseModule import BaseModule

__all__ = ["BaseModule"]
