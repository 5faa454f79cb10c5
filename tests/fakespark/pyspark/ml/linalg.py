class VectorUDT:
    """Marker type of vector columns in the fake schema."""
