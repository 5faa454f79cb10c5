class Column:
    def __init__(self, name, op=None):
        self.name, self.op = name, op


def col(name):
    return Column(name)


def unwrap_udt(c):
    return Column(c.name, "unwrap_udt")
