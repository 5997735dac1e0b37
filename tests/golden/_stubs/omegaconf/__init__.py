DictConfig = dict
