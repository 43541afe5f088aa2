from ..BaseModule import BaseModule


class Loss(BaseModule):
    pass
