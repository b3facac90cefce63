"""L2-regularised logistic regression of the reference (networks/logreg_model_titanic.py:4-29).

Host numpy model: P = 7 parameters per agent, nothing here is worth a kernel.
``calc_accuracy`` uses ``int`` where the reference used the removed ``np.int`` alias (:28)."""
import numpy as np


class LogRegTitanic:
    def __init__(self, dim, lr=5e-4, tau=1e-4):
        self.W = np.zeros(dim)
        self.lr = lr
        self.tau = tau

    def parameters(self):
        return self.W

    def _sigmoid(self, x):
        return 1.0 / (1.0 + np.exp(-x))

    def gradient(self, x_train, y_train, w=None):
        """-sum_j (y * sigmoid(-y * Xw)) . X[:, j] / n + tau * w   (:17-20).
        The reference's list comprehension re-evaluates y * sigmoid(-y * Xw) for each of the
        d columns; it is the same array every time, so it is formed once here and each column
        still gets its own np.dot on the strided column view, as the reference's does -- the
        same bits at a d-th of the matvecs and exponentials."""
        w = self.W if w is None else w
        r = y_train * self._sigmoid(-y_train * (x_train @ w))
        return -np.array([np.dot(r, x_train[:, j]) for j in range(x_train.shape[1])]) \
            / x_train.shape[0] + self.tau * w

    def loss(self, x, y, w=None):
        w = self.W if w is None else w
        return self.tau / 2 * np.sum(w ** 2) + -np.mean(np.log(self._sigmoid(y * (x @ w))))

    def fit(self, x_train, y_train):
        self.W -= self.lr * self.gradient(x_train, y_train)
        return self.loss(x_train, y_train)

    def calc_accuracy(self, x_test, y_test):
        test_predictions = (self._sigmoid(x_test @ self.W) >= 0.5).astype(int) * 2 - 1
        return np.mean(test_predictions == y_test)
