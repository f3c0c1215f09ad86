"""placeholder replaced below"""
def fuse_tensor_patterns(sinks, engine):
    return sinks, []
