class Mesh:
    pass


class MultiscaleMesh(Mesh):
    pass


def rotate_mesh(mesh, angle):
    raise NotImplementedError("stub")


def graph_from_mesh(mesh):  # import-only (utils/visualization.py)
    raise NotImplementedError("stub")


def remove_ghost_cells(*a, **k):  # import-only (utils/visualization.py)
    raise NotImplementedError("stub")
