"""cylon_amd.data"""
