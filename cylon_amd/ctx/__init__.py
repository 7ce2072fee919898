"""cylon_amd.ctx"""
