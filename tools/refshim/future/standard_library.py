def install_aliases():
    return None
