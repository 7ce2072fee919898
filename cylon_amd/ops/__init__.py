"""cylon_amd.ops"""
