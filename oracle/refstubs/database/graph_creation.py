class Mesh:
    pass


class MultiscaleMesh(Mesh):
    pass


def rotate_mesh(mesh, angle):
    raise NotImplementedError("stub")
