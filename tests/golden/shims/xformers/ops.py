"""Import-only stand-in (DenoiseNet_STWAtt_w_wo_ref_adaptor_cross_multi.py:13, unused)."""
