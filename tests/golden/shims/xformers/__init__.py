"""Import-only stand-in: the wo_ref denoiser imports xformers.ops but never calls it."""
