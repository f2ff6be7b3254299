"""minitorch (MI355X edition): the reference's minitorch operator surface on HIP/gfx950."""
