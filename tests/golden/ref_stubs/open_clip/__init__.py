def create_model_and_transforms(*a, **k):
    raise NotImplementedError("open_clip is not available offline")


def get_tokenizer(*a, **k):
    raise NotImplementedError("open_clip is not available offline")
