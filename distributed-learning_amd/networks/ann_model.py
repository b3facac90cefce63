"""4-layer MLP of the reference (networks/ann_model.py:4-45): 784 -> 150 ReLU -> 150 Tanh ->
150 ELU -> 10 for the MNIST shape.  Parameter registration order (fc1.w, fc1.b, ..., fc4.b) is
the flatten order ``Mixer`` uses (mixer.py:69), so the layout of a flattened agent row is the
same as the reference's."""
import torch.nn as nn


class ANNModel(nn.Module):
    def __init__(self, input_dim, hidden_dim, output_dim):
        super().__init__()
        self.fc1 = nn.Linear(input_dim, hidden_dim)
        self.relu1 = nn.ReLU()
        self.fc2 = nn.Linear(hidden_dim, hidden_dim)
        self.tanh2 = nn.Tanh()
        self.fc3 = nn.Linear(hidden_dim, hidden_dim)
        self.elu3 = nn.ELU()
        self.fc4 = nn.Linear(hidden_dim, output_dim)

    def forward(self, x):
        out = self.relu1(self.fc1(x))
        out = self.tanh2(self.fc2(out))
        out = self.elu3(self.fc3(out))
        return self.fc4(out)

    @staticmethod
    def param_shapes(input_dim, hidden_dim, output_dim):
        """Flattened-row layout: [(name, shape)] in registration order."""
        return [("fc1.weight", (hidden_dim, input_dim)), ("fc1.bias", (hidden_dim,)),
                ("fc2.weight", (hidden_dim, hidden_dim)), ("fc2.bias", (hidden_dim,)),
                ("fc3.weight", (hidden_dim, hidden_dim)), ("fc3.bias", (hidden_dim,)),
                ("fc4.weight", (output_dim, hidden_dim)), ("fc4.bias", (output_dim,))]
