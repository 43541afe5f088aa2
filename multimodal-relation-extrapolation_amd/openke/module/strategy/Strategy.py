from ..BaseModule import BaseModule


class Strategy(BaseModule):
    pass
