class Mutation:
    def __init__(self):
        pass
