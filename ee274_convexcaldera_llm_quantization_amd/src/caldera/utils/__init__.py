"""Drop-in mirror of the reference package layout (src.caldera.*)."""
