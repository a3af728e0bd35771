class ChebConv:  # noqa: D101 - unused by every shipped config
    pass


class TAGConv:
    pass


class GATConv:
    pass
